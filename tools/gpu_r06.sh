#!/bin/bash
# Round-6 GPU call, parameterised: TESTS (pytest node ids, may be empty),
# TRACE=1 (recurrence phase trace), BENCH (configs for bench.py lines, "" for
# none), TAG (output name suffix).  Every GPU step has its own time limit; the
# first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-x}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -s --timeout 300 --timeout-method thread \
    > gpurun_out/t_$T.log 2>&1
  rc=$?; grep -E "passed|failed|error" gpurun_out/t_$T.log | tail -3; [ $rc -eq 0 ] || { tail -40 gpurun_out/t_$T.log; exit $rc; }
fi
if [ "${TRACE:-0}" = 1 ]; then
  timeout -k 10 200 python -u tools/xg_trace.py > gpurun_out/trace_$T.txt 2>&1 || { tail -20 gpurun_out/trace_$T.txt; exit 1; }
  cat gpurun_out/trace_$T.txt | tail -14
fi
for C in $BENCH; do
  timeout -k 10 400 python -u bench.py --config $C --no-cpu-baseline --no-parity --steps ${STEPS:-20} --warmup 5 ${BARGS} \
    > gpurun_out/b_${C}_$T.json 2> gpurun_out/b_${C}_$T.err || { tail -20 gpurun_out/b_${C}_$T.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/b_${C}_$T.json'));r=d['roofline']
print('$C', d['ms_per_step'], r.get('kernel'), r.get('mean_launch_us'), r.get('us_per_time_step'), d.get('steps_stats'))"
done
