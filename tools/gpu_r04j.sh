#!/bin/bash
# round 4: A/B of the fused forward's partial-sum layout (ablib/head = previous commit)
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
for i in 1 2; do
  for v in half cur; do
    if [ $v = half ]; then L=$R/ablib/half/libasr_hip.so; else L=$R/pytorch_end2end_speech_recognition_amd/libasr_hip.so; fi
    ASR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --config ctc5x512 --steps 15 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/ab_${v}_$i.json 2> gpurun_out/ab_${v}_$i.err || { tail gpurun_out/ab_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${v}_$i.json'));r=d['roofline'];o=r['other_kernels'];print('$v', d['ms_per_step'], r['kernel'], r['mean_launch_us'], {k:v.get('mean_launch_us') for k,v in o.items() if 'lstm' in k})"
  done
done
