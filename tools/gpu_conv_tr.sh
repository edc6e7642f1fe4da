#!/bin/bash
# tap-resident conv: tests, standalone bench, vgg_hier A/B against the tap GEMM
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_tr_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/conv_tr_tests.log 2>&1; rc=$?
tail -15 gpurun_out/conv_tr_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/conv_bench.py > gpurun_out/conv_bench.txt 2>&1 || { tail -20 gpurun_out/conv_bench.txt; exit 1; }
cat gpurun_out/conv_bench.txt
timeout -k 10 300 python -u -m pytest tests/test_vgg.py tests/test_parity_pins_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "vgg" > gpurun_out/conv_tr_vgg_tests.log 2>&1 || { tail -30 gpurun_out/conv_tr_vgg_tests.log; exit 1; }
tail -3 gpurun_out/conv_tr_vgg_tests.log
for i in 1 2; do
  for v in 0 1; do
    ASR_VGG_TR=$v timeout -k 10 200 python -u bench.py --config vgg_hier --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0 > gpurun_out/vggtr_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/vggtr_$v.json'));print('ASR_VGG_TR=$v', d['ms_per_step'])"
  done
done
