#!/bin/bash
# 32-bit dropout hash (two elements per hash, integer thresholds): whole suite, A/B vs prev
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04z_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/r04z_tests.log | tail -8; [ $rc = 0 ] || exit 1
R=$(pwd)
for i in 1 2; do for c in vgg_hier ctc5x512 att4x320; do for v in prev cur; do
  if [ $v = prev ]; then L=$R/ablib/prev/libasr_hip.so; else L=$R/pytorch_end2end_speech_recognition_amd/libasr_hip.so; fi
  ASR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --config $c --steps 12 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/z_${c}_$v.json 2> gpurun_out/z_${c}_$v.err || { tail gpurun_out/z_${c}_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/z_${c}_$v.json'));print('$c $v', d['ms_per_step'])"
done; done; done
bash tools/gpu_ktrace.sh vgg_hier r04z > /dev/null || exit 1
grep -E "rw_" gpurun_out/r04z_kernel_stats_vgg_hier.txt | cut -c1-70,90-150
