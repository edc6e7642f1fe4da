#!/bin/bash
# round-5 end (c): kernel stats of the five configs, PMC traffic of ctc5x512 and vgg_hier
set -o pipefail
mkdir -p gpurun_out
for c in ctc5x512 timit2x320 att4x320 hybrid4x320 vgg_hier; do
  bash tools/gpu_ktrace.sh $c r05 > /dev/null || exit 1
  echo "$c: $(head -3 gpurun_out/r05_kernel_stats_$c.txt | tail -2 | cut -c1-60,90-140 | tr '\n' ' ')"
done
bash tools/gpu_pmc.sh r05 > /dev/null || exit 1
cat gpurun_out/r05_pmc_traffic.json | head -40
CONFIG=vgg_hier WORKLOAD=vgg_hier bash tools/gpu_pmc.sh r05_vgg > /dev/null || exit 1
timeout -k 10 300 python -u tools/gemm_bench.py > gpurun_out/r05_gemm_bench_bf16.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemm_f32_bench.py > gpurun_out/r05_gemm_bench_f32.txt 2>&1 || exit 1
cat gpurun_out/r05_gemm_bench_bf16.txt gpurun_out/r05_gemm_bench_f32.txt | grep -v amdgpu.ids
