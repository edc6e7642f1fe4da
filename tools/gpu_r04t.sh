#!/bin/bash
# VGG row passes back to one walker per lane: tests + vgg_hier kernel stats + A/B bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vgg_rows_gpu.py tests/test_parity_pins_gpu.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04t_tests.log; [ $rc = 0 ] || exit 1
bash tools/gpu_ktrace.sh vgg_hier r04t > /dev/null || exit 1
grep -E "rw_|c1_fwd" gpurun_out/r04t_kernel_stats_vgg_hier.txt | cut -c1-70,90-150
R=$(pwd)
for i in 1 2; do for v in head cur; do
  if [ $v = head ]; then L=$R/ablib/head/libasr_hip.so; export ASR_VGG_C1_RELU_P=0; else unset ASR_VGG_C1_RELU_P; L=$R/pytorch_end2end_speech_recognition_amd/libasr_hip.so; fi
  ASR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --config vgg_hier --steps 12 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/t_$v.json 2> gpurun_out/t_$v.err || { tail gpurun_out/t_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/t_$v.json'));print('vgg_hier $v', d['ms_per_step'])"
done; done
