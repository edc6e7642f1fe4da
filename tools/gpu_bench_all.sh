#!/bin/bash
# Every bench config once (default steps), for DESIGN.md numbers
set -o pipefail
mkdir -p gpurun_out
for C in ${CONFIGS:-ctc5x512 timit2x320 att4x320 hybrid4x320 vgg_hier}; do
  timeout -k 10 400 python -u bench.py --config $C ${EXTRA} > gpurun_out/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -20 gpurun_out/bench_$C.log; exit 1; }
  tail -1 gpurun_out/bench_$C.log | cut -c1-330
done
