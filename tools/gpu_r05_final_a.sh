#!/bin/bash
# round-5 end (a): the whole GPU suite and the smoke step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/r05_gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r05_gpu_tests.log | tail -5
[ $rc = 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r05_smoke.log; exit $rc
