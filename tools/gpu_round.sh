#!/bin/bash
# Round check: GPU test suite, smoke, then every bench config + kernel stats.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/round_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/round_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
for C in ${CONFIGS:-ctc5x512 timit2x320 att4x320 hybrid4x320 vgg_hier}; do
  timeout -k 10 400 python -u bench.py --config $C ${EXTRA} > gpurun_out/bench_$C.log 2>&1 || { echo "bench $C failed"; tail -20 gpurun_out/bench_$C.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_$C.log').read().strip().splitlines()[-1]);print('$C', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], (d.get('h2d') or {}).get('ms_per_step'), (d.get('parity') or {}).get('best_loss_rel_err_fp32'))"
done
if [ -n "$KTRACE" ]; then
  for C in $KTRACE; do bash tools/gpu_ktrace.sh $C ${TAG:-r03} || exit 1; done
fi
