#!/bin/bash
# round 5: backward recurrence interference from the side-stream GEMMs (ctc5x512)
set -o pipefail
mkdir -p gpurun_out
for v in "m3:ASR_OVERLAP_WGRAD=3" "m0x32:ASR_OVERLAP_WGRAD=0 ASR_XG_BWD_XU=32" "m0x16:ASR_OVERLAP_WGRAD=0 ASR_XG_BWD_XU=16" "m2:ASR_OVERLAP_WGRAD=2"; do
  n=${v%%:*}; e=${v#*:}
  env $e timeout -k 10 240 python -u bench.py --config ctc5x512 --steps 15 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/intf_$n.json 2> gpurun_out/intf_$n.err || { tail -3 gpurun_out/intf_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/intf_$n.json'));r=d['roofline'];o=r.get('other_kernels',{});print('$n', d['ms_per_step'], r.get('kernel')[:40], r['mean_launch_us'], [ (k[:30], v['mean_launch_us']) for k,v in o.items() if 'lstm' in k])"
done
