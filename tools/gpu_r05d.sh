#!/bin/bash
# round 5: fault-era build (001db35) variants: tanh-gate decode without a branch; no packed FP32
set -o pipefail
mkdir -p gpurun_out
cd oldtree
run() {  # name, env...
  local n=$1; shift
  env "$@" DIAG_DH=0 DIAG_REPS=3 timeout -k 10 300 python -u tools/cores_locate.py mode2 > ../gpurun_out/r05_old_$n.log 2>&1
  local rc=$?
  echo "== $n rc=$rc"
  grep "== \|call [01] dG\|reproducible" ../gpurun_out/r05_old_$n.log | sed 's/unit slices.*at the earliest/... earliest/' | cut -c1-250
  return $rc
}
run nobr ASR_LIB_PATH=var/nobr/libasr_hip.so && \
run nopk ASR_LIB_PATH=var/nopk/libasr_hip.so
