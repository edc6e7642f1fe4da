#!/bin/bash
# decoder tests, then att4x320 with the decoder's internal W_dec products on the f32 fast kernel vs the generic one
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_attdec_persist.py tests/test_parity_pins_gpu.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/wdec_tests.log 2>&1
rc=$?; tail -1 gpurun_out/wdec_tests.log; [ $rc = 0 ] || exit 1
for m in 1 0 1 0; do
  ASR_GEMM_F32FAST=$m timeout -k 10 300 python -u bench.py --config att4x320 --no-cpu-baseline --no-parity > gpurun_out/wdec_$m.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/wdec_$m.json'));print('f32fast=$m', d['ms_per_step'])"
done
