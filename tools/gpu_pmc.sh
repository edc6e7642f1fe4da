#!/bin/bash
# PMC passes for the bench's HBM traffic (one counter group per pass, no tracing
# beside --pmc), then the kernel-trace stats of the same command.
#   bash tools/gpu_pmc.sh <round-tag>
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --config ${CONFIG:-ctc5x512} --steps 2 --warmup 1 --no-cpu-baseline"
rm -rf $OUT/pmc_fetch $OUT/pmc_write $OUT/ktrace
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -- python3 $BENCH > $OUT/pmc_fetch.log 2>&1 || { echo "fetch pass failed"; tail -20 $OUT/pmc_fetch.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -- python3 $BENCH > $OUT/pmc_write.log 2>&1 || { echo "write pass failed"; tail -20 $OUT/pmc_write.log; exit 1; }
python3 $R/tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write ${WORKLOAD:-librispeech100h_char_ctc_blstm5x512} > $OUT/${TAG}_pmc_traffic.json || exit 1
cat $OUT/${TAG}_pmc_traffic.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -- python3 $R/bench.py --config ${CONFIG:-ctc5x512} --steps 5 --warmup 2 --no-cpu-baseline > $OUT/ktrace.log 2>&1 || { echo "trace pass failed"; tail -20 $OUT/ktrace.log; exit 1; }
tail -1 $OUT/ktrace.log
KT=$(find $OUT/ktrace -name '*kernel_trace.csv' -print -quit)
python3 $R/profiles/kstats.py $KT > $OUT/${TAG}_kernel_stats.txt && head -25 $OUT/${TAG}_kernel_stats.txt
