#!/bin/bash
# GPU suite, then att4x320 / vgg_hier with the GEMM operand staging in one launch vs per operand
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/stage_tests.log 2>&1
rc=$?; tail -1 gpurun_out/stage_tests.log; [ $rc = 0 ] || exit 1
for c in att4x320 vgg_hier; do
  for m in 1 0 1 0; do
    ASR_GEMM_STAGE_MULTI=$m timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-parity > gpurun_out/stage_${c}_${m}.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/stage_${c}_${m}.json'));print('$c multi=$m', d['ms_per_step'])"
  done
done
