#!/bin/bash
# A/B: fused bias gradients vs separate column-sum pass, loss trajectory + speed
set -o pipefail
mkdir -p gpurun_out
for F in 0 1; do
  ASR_BIAS_FUSED=$F timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bias_ab_$F.log 2>&1 || { tail -20 gpurun_out/bias_ab_$F.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bias_ab_$F.log').read().strip().splitlines()[-1]); print('fused=$F', d['value'], d['ms_per_step'], d['loss_last'])"
done
