#!/bin/bash
# round 5: fault-era build (001db35) variants: cell lanes transposed, inputs one step ahead
set -o pipefail
mkdir -p gpurun_out
cd oldtree
run() {  # name, env...
  local n=$1; shift
  env "$@" DIAG_DH=0 DIAG_REPS=3 timeout -k 10 300 python -u tools/cores_locate.py mode2 > ../gpurun_out/r05_old_$n.log 2>&1
  local rc=$?
  echo "== $n rc=$rc"
  grep "== \|call [01] dG\|reproducible" ../gpurun_out/r05_old_$n.log | cut -c1-260
  return $rc
}
run cellT ASR_LIB_PATH=var/cellT/libasr_hip.so && \
run pref1 ASR_LIB_PATH=var/pref1/libasr_hip.so && \
run head3 ASR_XG_BWD_IO=0
