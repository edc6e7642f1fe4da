#!/bin/bash
# lattice kernel durations, single- vs multi-wave (+ CTC tests)
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  ASR_CTC_LATTICE_MW=$m timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lat$m -- python3 $R/tools/ctc_bench.py > $R/gpurun_out/lat$m.log 2>&1 || { tail $R/gpurun_out/lat$m.log; exit 1; }
  KT=$(find $R/gpurun_out/lat$m -name '*kernel_trace.csv' -print -quit)
  echo "== mw=$m"; python3 $R/profiles/kstats.py $KT | grep -i -E "lattice|ctc" | cut -c1-40,90-150
done
