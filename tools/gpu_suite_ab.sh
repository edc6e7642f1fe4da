#!/bin/bash
# full GPU suite, then an interleaved A/B of the archived tree (ab/old) against this one
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/suite.log 2>&1; rc=$?
tail -2 gpurun_out/suite.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/suite.log | head -20; exit $rc; }
for C in ${CONFIGS:-hybrid4x320}; do
  for i in 1 2; do
    for nv in head=ab/old new=.; do
      n=${nv%%=*}; p=${nv#*=}
      (cd $p && timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0) > gpurun_out/sab_${C}_$n.json 2>/dev/null || exit 1
      python -c "import json;d=json.load(open('gpurun_out/sab_${C}_$n.json'));print('$C $n', d['ms_per_step'])"
    done
  done
done
