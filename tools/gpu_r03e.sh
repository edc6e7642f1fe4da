#!/bin/bash
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u tools/buckets_diag.py trace 2 2>&1 | grep -v amdgpu.ids > gpurun_out/r03e_$name.log; local rc=$?
  echo "== $name rc=$rc"; grep "dx\|diag" gpurun_out/r03e_$name.log
  return $rc
}
run nosplit DIAG_WHH=0.03 ASR_GEMM_NOSPLIT=1 && run nosplit_b DIAG_WHH=0.03 ASR_GEMM_NOSPLIT=1 && run nosplit_scr DIAG_WHH=0.03 ASR_GEMM_NOSPLIT=1 ASR_DIAG_WGRAD_SCRATCH=1
