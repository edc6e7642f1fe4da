#!/bin/bash
# one GPU call: selected tests ($TESTS), then whole-step A/B of $VARIANTS (tools/gpu_ab.sh)
set -o pipefail
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/round_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/round_tests.log; exit 1; }
  tail -1 gpurun_out/round_tests.log
fi
bash tools/gpu_ab.sh 2>&1 | tee gpurun_out/round_ab.log
