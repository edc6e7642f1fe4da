#!/bin/bash
# round 5: bf16 CTC head gradient -- blocks (rows per block) A/B under rocprof
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for nb in 512 1024 2048; do
rm -rf gpurun_out/r_prof_$nb
ASR_CTC_BIAS_BLOCKS=$nb HEAD_MODES=bf16 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r_prof_$nb -- python3 tools/ctc_head_bench.py > gpurun_out/r_head_$nb.log 2>&1
rc=$?; echo "blocks $nb: $(grep 'us / iteration' gpurun_out/r_head_$nb.log)"; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/r_prof_$nb -name "*kernel_stats.csv" | head -1); python3 -c "
import csv
r=list(csv.DictReader(open('$f')))
for x in r:
  if 'ctc_grad' in x['Name'] or 'colsum' in x['Name']: print('   %-50s %6s %10.1f' % (x['Name'][:50], x['Calls'], float(x['AverageNs'])/1000))"
done
