#!/bin/bash
# ring GEMM vs two-buffer 8-wave kernel at the 5x512 shapes; ablations at dX
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k 8wave --timeout 120 --timeout-method thread 2>&1 | tail -1
for v in 0 1 0 1; do
  ASR_GEMM_LIB=0 ASR_GEMM_8R=$v timeout -k 10 60 python -u tools/gemm_bench.py 2>&1 | grep TF | sed "s/^/8R=$v /"
done
for v in 11 12; do
  ASR_GEMM_LIB=0 ASR_GEMM_8R=$v GEMM_BENCH_ONLY=dX timeout -k 10 60 python -u tools/gemm_bench.py 2>&1 | grep TF | sed "s/^/8R=$v /"
done
