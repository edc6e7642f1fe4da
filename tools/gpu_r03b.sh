#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_pins_gpu.py tests/test_model_ctc.py tests/test_grad_buckets_gpu.py tests/test_step_hygiene_gpu.py -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "vs float64|passed|failed|Error" gpurun_out/r03b_tests.log | head -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/buckets_diag.py 2 > gpurun_out/r03b_diag.log 2>&1
rc2=$?; echo "diag rc=$rc2"; cat gpurun_out/r03b_diag.log | grep -v amdgpu.ids | head -60
