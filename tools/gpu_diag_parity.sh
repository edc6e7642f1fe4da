#!/bin/bash
# vgg_hier fp32 parity under single switches
set -o pipefail
mkdir -p gpurun_out
run() { env "$@" timeout -k 10 300 python -u tools/diag_parity.py 2>&1 | grep -v amdgpu.ids | tail -1; }
run DIAG_X=1 || exit 1
run ASR_LSTM_XG32=0 || exit 1
run ASR_GEMM_F32FAST=0 || exit 1
run ASR_CTC_LSE_EPI=0 || exit 1
run ASR_LSTM_XG32=0 ASR_GEMM_F32FAST=0 ASR_CTC_LSE_EPI=0 || exit 1
