#!/bin/bash
# GPU check: parity tests, then the default bench line (+ optional extra configs in $CONFIGS).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
for C in ${CONFIGS}; do
  timeout -k 10 400 python -u bench.py --config $C > gpurun_out/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -30 gpurun_out/bench_$C.log; exit 1; }
  tail -1 gpurun_out/bench_$C.log
done
