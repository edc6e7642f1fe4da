#!/bin/bash
# full GPU suite (one process) + smoke; log under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/suite_${1:-x}.log 2>&1
rc=$?
tail -5 gpurun_out/suite_${1:-x}.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_${1:-x}.log 2>&1
rc=$?
tail -2 gpurun_out/smoke_${1:-x}.log
exit $rc
