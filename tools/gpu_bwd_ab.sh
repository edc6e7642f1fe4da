#!/bin/bash
# backward-recurrence A/B: parity tests of the BLSTM layer, whole-step A/B of $VARIANTS, phase trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encoder_gpu.py tests/test_recurrence_full.py tests/test_model_ctc.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bwd_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/bwd_tests.log; exit 1; }
tail -1 gpurun_out/bwd_tests.log
STEPS=${STEPS:-10} bash tools/gpu_ab.sh 2>&1 | tee gpurun_out/bwd_ab.log
timeout -k 10 120 python -u tools/xg_trace.py > gpurun_out/xg_trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/xg_trace.log; exit 1; }
cat gpurun_out/xg_trace.log
