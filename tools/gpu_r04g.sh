#!/bin/bash
# round 4: 32 units per backward work-group (half the CUs at 5x512) + mode-3 overlap
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_recurrence_full.py tests/test_grad_buckets_gpu.py -s -k "units or full_shape or buckets" > gpurun_out/r04g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "units per|full-shape|PASS|FAIL|Error|passed|failed" gpurun_out/r04g_tests.log | cut -c1-400 | tail -20
[ $rc = 0 ] || exit 1
for i in 1 2; do
  for xu in 16 auto; do
    ASR_XG_BWD_XU=$xu timeout -k 10 200 python -u bench.py --config ctc5x512 --steps 15 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/xu_${xu}_$i.json 2> gpurun_out/xu_${xu}_$i.err || { tail gpurun_out/xu_${xu}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/xu_${xu}_$i.json'));r=d['roofline'];o=r['other_kernels'];print('$xu', d['ms_per_step'], r['kernel'], r['mean_launch_us'], {k:v.get('mean_launch_us') for k,v in o.items() if 'lstm' in k})"
  done
done
