#!/bin/bash
# round 5: fp32 att4x320 kernel breakdown
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/s_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s_prof -- python3 bench.py --config att4x320 --precision fp32 --steps 5 --warmup 2 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/s_att.log 2>&1
rc=$?; tail -1 gpurun_out/s_att.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/s_prof -name "*kernel_stats.csv" | head -1); python3 -c "
import csv
r=list(csv.DictReader(open('$f')))
tot=sum(float(x['TotalDurationNs']) for x in r)
print('total kernel ms per step', tot/1e6/7)
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:25]: print('%-70s %6s %9.1f %6.2f' % (x['Name'][:70], x['Calls'], float(x['AverageNs'])/1000, float(x['TotalDurationNs'])/1e6/7))"
