#!/bin/bash
# Round-3 check: GPU test suite, then (only if pytest ended normally, pass or
# fail) one short bench run with the H2D and parity legs.
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r03_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/r03_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r03_bench.log 2>&1
rc2=$?
echo "bench rc=$rc2"
tail -c 3000 gpurun_out/r03_bench.log
exit $rc2
