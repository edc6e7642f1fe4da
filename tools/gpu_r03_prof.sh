#!/bin/bash
# Round-3 profiles: kernel stats of the attention / hybrid / VGG configs, the
# GEMM bench at the 5x512 shapes and the standalone CTC bench.
set -o pipefail
mkdir -p gpurun_out
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 200 python -u tools/gemm_bench.py > gpurun_out/r03_gemm_bench.txt 2>&1 || { tail -20 gpurun_out/r03_gemm_bench.txt; exit 1; }
cat gpurun_out/r03_gemm_bench.txt
timeout -k 10 120 python -u tools/ctc_bench.py > gpurun_out/r03_ctc_bench.jsonl 2>&1 || { tail -20 gpurun_out/r03_ctc_bench.jsonl; exit 1; }
cat gpurun_out/r03_ctc_bench.jsonl
for C in ${KTRACE:-att4x320 hybrid4x320 vgg_hier}; do bash tools/gpu_ktrace.sh $C r03 || exit 1; done
