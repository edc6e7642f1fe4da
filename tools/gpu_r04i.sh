#!/bin/bash
# round 4: forward recurrence phase trace + ctc5x512 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/xg_trace.py 2>&1 | tail -12 || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config ctc5x512 --steps 15 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/fw_$i.json 2> gpurun_out/fw_$i.err || { tail gpurun_out/fw_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/fw_$i.json'));r=d['roofline'];o=r['other_kernels'];print(d['ms_per_step'], r['kernel'], r['mean_launch_us'], {k:v.get('mean_launch_us') for k,v in o.items() if 'lstm' in k})"
done
