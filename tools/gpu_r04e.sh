#!/bin/bash
# round 4 baseline: ctc5x512 bench line (roofline rows) + its kernel stats, CTC bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config ctc5x512 --no-cpu-baseline > gpurun_out/r04e_ctc5x512.json 2> gpurun_out/r04e_ctc5x512.err || { tail -20 gpurun_out/r04e_ctc5x512.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r04e_ctc5x512.json'))
r=d['roofline']; print(d['ms_per_step'], r['kernel'], r['mean_launch_us'], r.get('us_per_time_step'), r['frac'])
for k,v in sorted(r['other_kernels'].items(), key=lambda kv:-kv[1].get('share_of_timed_kernel_time',0))[:14]: print('  ', k, v.get('mean_launch_us', v.get('mean_call_us')), v.get('launches'), v.get('achieved'), v.get('unit'), v.get('share_of_timed_kernel_time'))
"
STEPS=5 bash tools/gpu_ktrace.sh ctc5x512 r04 || exit 1
timeout -k 10 120 python -u tools/ctc_bench.py > gpurun_out/r04_ctc_bench.jsonl 2>&1 || { tail -20 gpurun_out/r04_ctc_bench.jsonl; exit 1; }
cat gpurun_out/r04_ctc_bench.jsonl
