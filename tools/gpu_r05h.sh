#!/bin/bash
# round 5: backward cell precompute A/B + recurrence parity
set -o pipefail
mkdir -p gpurun_out
tools/gpu_abcfg.sh pre 2 "ctc5x512 timit2x320" pre=ablib/head/libasr_hip.so nopre=ablib/nopre/libasr_hip.so || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_recurrence_full.py tests/test_coresidency_gpu.py > gpurun_out/r05h_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05h_tests.log
exit $rc
