#!/bin/bash
# Every bench config once (short), for DESIGN.md numbers
set -o pipefail
mkdir -p gpurun_out
for C in ctc5x512 att4x320 hybrid4x320 vgg_hier; do
  timeout -k 10 300 python -u bench.py --config $C --steps ${STEPS:-10} --warmup 3 ${EXTRA} > gpurun_out/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -20 gpurun_out/bench_$C.log; exit 1; }
  tail -1 gpurun_out/bench_$C.log | cut -c1-420
done
