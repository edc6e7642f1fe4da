#!/bin/bash
# round 5: co-residency fault -- does HEAD still reproduce (mode 2, 5x512), and
# the three non-instrumenting variants of VERDICT r04 item 1
set -o pipefail
mkdir -p gpurun_out
run() {  # name, env...
  local n=$1; shift
  env "$@" DIAG_DH=0 DIAG_REPS=2 timeout -k 10 300 python -u tools/cores_locate.py mode2 > gpurun_out/r05_loc_$n.log 2>&1
  local rc=$?
  echo "== $n rc=$rc"
  grep "== \|call [01] dG\|reproducible" gpurun_out/r05_loc_$n.log | cut -c1-230
  return $rc
}
run head ASR_XG_BWD_IO=0 && \
run st16off ASR_XG_DG_ST16=0 && \
run cellT ASR_LIB_PATH=ablib/cellT/libasr_hip.so && \
run pref1 ASR_LIB_PATH=ablib/pref1/libasr_hip.so
