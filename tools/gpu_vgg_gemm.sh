#!/bin/bash
# VGG A/B (tests + vgg_hier against ab/old), then the GEMM PMC passes.
set -o pipefail
bash tools/gpu_vgg_ab.sh || exit $?
bash tools/gemm_pmc_r03.sh > gpurun_out/gemm_pmc_r03.txt 2>&1 || { tail -5 gpurun_out/gemm_pmc_r03.txt; exit 1; }
tail -60 gpurun_out/gemm_pmc_r03.txt
