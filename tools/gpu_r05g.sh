#!/bin/bash
# round 5: co-residency tests (modes 2 / 3 vs 0 bitwise, side traffic), CTC, dropout RNG, buckets
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_coresidency_gpu.py tests/test_dropout_rng_gpu.py tests/test_grad_buckets_gpu.py \
  tests/test_ctc_gpu.py tests/test_model_ctc.py > gpurun_out/r05g_tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/r05g_tests.log | tail -50
exit $rc
