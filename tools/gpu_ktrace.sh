#!/bin/bash
# kernel-trace stats of one bench config: bash tools/gpu_ktrace.sh <config> <tag>
set -o pipefail
C=${1:-ctc5x512}; TAG=${2:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT && rm -rf $OUT/ktrace_$C
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace_$C -- python3 $R/bench.py --config $C --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $OUT/ktrace_$C.log 2>&1 || { echo "trace failed"; tail -20 $OUT/ktrace_$C.log; exit 1; }
tail -1 $OUT/ktrace_$C.log | cut -c1-300
KT=$(find $OUT/ktrace_$C -name '*kernel_trace.csv' -print -quit)
python3 $R/profiles/kstats.py $KT > $OUT/${TAG}_kernel_stats_$C.txt && head -30 $OUT/${TAG}_kernel_stats_$C.txt
