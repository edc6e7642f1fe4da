#!/bin/bash
# CTC row order A/B (ASR_CTC_ORDER 0..3) on the standalone bench, CTC tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ctc_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ctc_tests.log 2>&1 || { tail -20 gpurun_out/ctc_tests.log; exit 1; }
tail -1 gpurun_out/ctc_tests.log
for r in 1 2; do
  for o in 0 2 1 3; do
    ASR_CTC_ORDER=$o timeout -k 10 120 python -u tools/ctc_bench.py > gpurun_out/ctc_order_$o.jsonl 2>/dev/null || exit 1
    python -c "import json;d=[json.loads(l) for l in open('gpurun_out/ctc_order_$o.jsonl') if l.startswith('{')];print('order $o', d[0]['us_per_call'], d[0]['frac'])"
  done
done
