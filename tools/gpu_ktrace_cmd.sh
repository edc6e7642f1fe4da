#!/bin/bash
# kernel-trace stats of an arbitrary python script: bash tools/gpu_ktrace_cmd.sh <tag> <script> [args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT && rm -rf $OUT/kt_$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$TAG -- python3 $R/$@ > $OUT/kt_$TAG.log 2>&1 || { echo "trace failed"; tail -20 $OUT/kt_$TAG.log; exit 1; }
KT=$(find $OUT/kt_$TAG -name '*kernel_trace.csv' -print -quit)
python3 $R/profiles/kstats.py $KT > $OUT/kstats_$TAG.txt && head -20 $OUT/kstats_$TAG.txt
