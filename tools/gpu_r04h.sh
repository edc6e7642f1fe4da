#!/bin/bash
# round 4: bf16 hand-off between BLSTM layers (no f32 y, no staging pass)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_model_ctc.py tests/test_encoder_gpu.py -s > gpurun_out/r04h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/r04h_tests.log | cut -c1-300 | tail -12
[ $rc = 0 ] || exit 1
for i in 1 2; do
  for ho in 0 1; do
    ASR_BF16_HANDOFF=$ho timeout -k 10 200 python -u bench.py --config ctc5x512 --steps 15 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/ho_${ho}_$i.json 2> gpurun_out/ho_${ho}_$i.err || { tail gpurun_out/ho_${ho}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ho_${ho}_$i.json'));r=d['roofline'];o=r['other_kernels'];print('$ho', d['ms_per_step'], r['kernel'], r['mean_launch_us'], {k:v.get('mean_launch_us') for k,v in o.items() if 'lstm' in k or 'conv' in k})"
  done
done
