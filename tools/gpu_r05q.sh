#!/bin/bash
# round 5: CTC head kernels (rocprof stats) after the bf16 gradient's load batching
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_ctc_gpu.py tests/test_model_ctc.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/q_tests.log 2>&1
rc=$?; tail -2 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/q_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/q_prof -- python3 tools/ctc_head_bench.py > gpurun_out/q_head.log 2>&1
rc=$?; grep "us / iteration" gpurun_out/q_head.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/q_prof -name "*kernel_stats.csv" | head -1); python3 -c "
import csv
r=list(csv.DictReader(open('$f')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:14]: print('%-60s %6s %10.1f' % (x['Name'][:60], x['Calls'], float(x['AverageNs'])/1000))"
