#!/bin/bash
# decoder-side weight gradients beside the encoder's top recurrence: tests + A/B
set -o pipefail
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_attention_prod.py tests/test_model_ctc.py tests/test_model_attention.py tests/test_attdec_persist.py tests/test_step_hygiene_gpu.py tests/test_grad_buckets_gpu.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04dw_tests.log 2>&1
rc=$?; [ $rc = 0 ] || exit 1
for i in 1 2 3 4; do for c in att4x320 hybrid4x320; do for m in 0 1; do
  ASR_DEC_WGRAD_SIDE=$m timeout -k 10 200 python -u bench.py --config $c --steps 12 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/dw_${c}_$m.json 2> gpurun_out/dw_${c}_$m.err || { tail gpurun_out/dw_${c}_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/dw_${c}_$m.json'));print('$c dec_side=$m', d['ms_per_step'])"
done; done; done
