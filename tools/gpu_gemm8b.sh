#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
ASR_GEMM_LIB=0 timeout -k 10 120 python -u tools/gemm_bench.py > gpurun_out/gb.log 2>&1; cat gpurun_out/gb.log | grep TF; bash tools/gemm8_pmc.sh
