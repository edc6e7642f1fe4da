#!/bin/bash
# round 4: row-blocked VGG element-wise passes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_vgg_rows_gpu.py tests/test_parity_pins_gpu.py tests/test_conv_tr_gpu.py -s > gpurun_out/r04n_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed|assert" gpurun_out/r04n_tests.log | cut -c1-300 | tail -16
[ $rc = 0 ] || exit 1
for i in 1 2; do
  for v in 0 1; do
    ASR_VGG_ROWS=$v timeout -k 10 200 python -u bench.py --config vgg_hier --steps 12 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/vr_${v}_$i.json 2> gpurun_out/vr_${v}_$i.err || { tail gpurun_out/vr_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/vr_${v}_$i.json'));print('$v', d['ms_per_step'])"
  done
done
bash tools/gpu_ktrace.sh vgg_hier r04rows > /dev/null && grep -E "post_|apply|moments|rw_" gpurun_out/r04rows_kernel_stats_vgg_hier.txt | cut -c1-60,90-140
