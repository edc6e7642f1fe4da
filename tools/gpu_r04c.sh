#!/bin/bash
# round 4: mode 3 (side-stream weight gradients on the CUs the recurrence leaves free)
set -o pipefail
mkdir -p gpurun_out
DIAG_REPS=3 DIAG_H=320 DIAG_L=4 timeout -k 10 300 python -u tools/cores_locate.py mode3 mode2 > gpurun_out/locate6.log 2>&1
echo "locate rc=$?"
grep "== \|call . dG" gpurun_out/locate6.log | cut -c1-160 | head -40
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_grad_buckets_gpu.py tests/test_step_hygiene_gpu.py tests/test_model_ctc.py > gpurun_out/r04c_tests.log 2>&1
echo "tests rc=$?"
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r04c_tests.log | tail -40
