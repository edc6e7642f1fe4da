set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_attention_prod.py tests/test_recurrence_full.py tests/test_model_ctc.py -m gpu -v -s --timeout 150 --timeout-method thread > gpurun_out/new_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error|full-shape|first 48" gpurun_out/new_tests.log | head -40
exit $rc
