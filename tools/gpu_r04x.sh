#!/bin/bash
# pipelined dX mode 2 (outer rows on the compute stream, middle beside the recurrence)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_dx_pipeline_gpu.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04x_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04x_tests.log; [ $rc = 0 ] || exit 1
for i in 1 2; do for c in ctc5x512 att4x320 timit2x320 vgg_hier; do for m in 0 2; do
  ASR_DX_PIPE=$m timeout -k 10 200 python -u bench.py --config $c --steps 12 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/x_${c}_$m.json 2> gpurun_out/x_${c}_$m.err || { tail gpurun_out/x_${c}_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/x_${c}_$m.json'));print('$c pipe=$m', d['ms_per_step'])"
done; done; done
