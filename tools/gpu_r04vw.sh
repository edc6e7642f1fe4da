#!/bin/bash
# VGG conv weight gradients on a side stream: tests + vgg_hier A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vgg_rows_gpu.py tests/test_parity_pins_gpu.py tests/test_conv_tr_gpu.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04vw_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|^E " gpurun_out/r04vw_tests.log | tail -6; [ $rc = 0 ] || exit 1
for i in 1 2 3; do for m in 0 1; do
  ASR_VGG_WGRAD_SIDE=$m timeout -k 10 200 python -u bench.py --config vgg_hier --steps 12 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/vw_$m.json 2> gpurun_out/vw_$m.err || { tail gpurun_out/vw_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/vw_$m.json'));print('vgg_hier wgrad_side=$m', d['ms_per_step'])"
done; done
