#!/bin/bash
# persistent decoder forward: A/B parity tests, then the attention tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attdec_persist.py -m gpu -v -x -s --timeout 120 --timeout-method thread > gpurun_out/pd_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert|prod|ragged" gpurun_out/pd_tests.log | head -30
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest ${PD_MORE:-tests/test_attention_prod.py tests/test_layer_boundaries_gpu.py tests/test_model_attention.py} -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/pd_more.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" gpurun_out/pd_more.log | head -40
exit $rc
