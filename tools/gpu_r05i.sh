#!/bin/bash
# round 5: pinned backward precompute: trace + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/xg_trace.py > gpurun_out/r05_xg_trace3.log 2>&1 || exit 1
grep -A5 "^backward" gpurun_out/r05_xg_trace3.log
tools/gpu_abcfg.sh pre2 2 "ctc5x512 timit2x320" pre=ablib/head/libasr_hip.so nopre=ablib/nopre/libasr_hip.so
