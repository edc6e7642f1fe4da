#!/bin/bash
# 8-wave GEMM: exactness tests, then throughput at the 5x512 shapes (library / 8-wave / 128x128)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -2 gpurun_out/gemm_tests.log
timeout -k 10 120 python -u tools/gemm_bench.py && \
ASR_GEMM_LIB=0 timeout -k 10 120 python -u tools/gemm_bench.py && \
ASR_GEMM_LIB=0 ASR_GEMM_8W=0 timeout -k 10 120 python -u tools/gemm_bench.py
