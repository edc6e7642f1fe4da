#!/bin/bash
# round 5: does the fault-era build (commit 001db35, the one locate2 ran) still
# reproduce on today's boxes?  oldtree/ = that commit's package + locator
set -o pipefail
mkdir -p gpurun_out
cd oldtree
run() {  # name, env...
  local n=$1; shift
  env "$@" DIAG_DH=0 DIAG_REPS=3 timeout -k 10 300 python -u tools/cores_locate.py mode2 > ../gpurun_out/r05_old_$n.log 2>&1
  local rc=$?
  echo "== $n rc=$rc"
  grep "== \|call [01] dG\|reproducible" ../gpurun_out/r05_old_$n.log | cut -c1-330
  return $rc
}
run head ASR_XG_BWD_IO=0 && \
run st16off ASR_XG_DG_ST16=0 && \
run head2 ASR_XG_BWD_IO=0
cd ..
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_ctc_gpu.py > gpurun_out/r05b_ctc_tests.log 2>&1
echo "ctc tests rc=$?"
grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/r05b_ctc_tests.log | tail -30
