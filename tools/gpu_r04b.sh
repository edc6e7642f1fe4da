#!/bin/bash
# round 4: dh-level co-residency localisation + the replayed bf16 VGG pins
set -o pipefail
mkdir -p gpurun_out
DIAG_REPS=2 timeout -k 10 300 python -u tools/cores_locate.py mode2 > gpurun_out/locate2.log 2>&1
echo "locate rc=$?"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_parity_pins_gpu.py tests/test_step_hygiene_gpu.py -s -k "vgg or retry" > gpurun_out/r04b_tests.log 2>&1
echo "tests rc=$?"
grep -v Warning gpurun_out/locate2.log | grep -v amdgpu.ids | grep -v "side_ent\|warnings.warn" | grep -v " dG: " | head -60
grep -E "PASS|FAIL|Error|error|bf16 VGG|passed|failed" gpurun_out/r04b_tests.log | tail -30
