#!/bin/bash
# pooled-grid VGG backward (ASR_VGG_POOL_WALK): tests, vgg_hier A/B, kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vgg_rows_gpu.py tests/test_parity_pins_gpu.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04p2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04p2_tests.log; [ $rc = 0 ] || exit 1
for i in 1 2; do for m in 0 1; do
  ASR_VGG_POOL_WALK=$m timeout -k 10 200 python -u bench.py --config vgg_hier --steps 12 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/p2_$m.json 2> gpurun_out/p2_$m.err || { tail gpurun_out/p2_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/p2_$m.json'));print('vgg_hier pool_walk=$m', d['ms_per_step'])"
done; done
bash tools/gpu_ktrace.sh vgg_hier r04p2 > /dev/null || exit 1
grep -E "rw_" gpurun_out/r04p2_kernel_stats_vgg_hier.txt | cut -c1-70,90-150
