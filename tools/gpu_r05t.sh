#!/bin/bash
# round 5: fp32 persistent decoder passes -- tests, fp32 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attdec_persist.py tests/test_attention_prod.py tests/test_model_attention.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/t_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t_tests.log; [ $rc -eq 0 ] || exit $rc
for c in att4x320 hybrid4x320; do
  timeout -k 10 300 python -u bench.py --config $c --precision fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/t_$c.json 2> gpurun_out/t_$c.err || { tail -3 gpurun_out/t_$c.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/t_$c.json'));r=d['roofline']
print('$c fp32', d['ms_per_step'], r['kernel'], r['mean_launch_us'], [(k[:30], v.get('mean_launch_us'), v.get('launches')) for k,v in r.get('other_kernels',{}).items()])"
done
