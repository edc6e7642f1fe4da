#!/bin/bash
# round 4: co-residency localisation + new pins (saturated packed gates, fused CTC head)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/cores_locate.py > gpurun_out/locate.log 2>&1
echo "locate rc=$?"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_recurrence_full.py tests/test_ctc_gpu.py -s > gpurun_out/r04a_tests.log 2>&1
echo "tests rc=$?"
grep -v Warning gpurun_out/locate.log | grep -v amdgpu.ids | tail -90
grep -E "PASS|FAIL|Error|error|saturated|passed|failed" gpurun_out/r04a_tests.log | tail -30
