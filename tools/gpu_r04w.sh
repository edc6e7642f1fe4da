#!/bin/bash
# VGG backward row pass with its BN parameters in LDS (8 waves / SIMD): tests, kernel stats, A/B vs prev
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vgg_rows_gpu.py tests/test_parity_pins_gpu.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04w_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04w_tests.log; [ $rc = 0 ] || exit 1
R=$(pwd)
for i in 1 2; do for v in prev cur; do
  if [ $v = prev ]; then L=$R/ablib/prev/libasr_hip.so; else L=$R/pytorch_end2end_speech_recognition_amd/libasr_hip.so; fi
  ASR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --config vgg_hier --steps 12 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/w_$v.json 2> gpurun_out/w_$v.err || { tail gpurun_out/w_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/w_$v.json'));print('vgg_hier $v', d['ms_per_step'])"
done; done
bash tools/gpu_ktrace.sh vgg_hier r04w > /dev/null || exit 1
grep -E "rw_" gpurun_out/r04w_kernel_stats_vgg_hier.txt | cut -c1-70,90-150
