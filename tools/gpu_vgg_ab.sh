#!/bin/bash
# VGG path change: the VGG / conv / hierarchical GPU tests, then an interleaved
# A/B of ab/libasr_hip_head.so against the working tree on vgg_hier
set -o pipefail
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] && rc=0 || { timeout -k 10 500 python -u -m pytest tests/test_vgg.py tests/test_conv_tr_gpu.py tests/test_hierarchical.py tests/test_parity_pins_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/vgg_ab_tests.log 2>&1; rc=$?; }
tail -4 gpurun_out/vgg_ab_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for nv in head=ab/old new=.; do
    n=${nv%%=*}; p=${nv#*=}
    (cd $p && timeout -k 10 200 python -u bench.py --config vgg_hier --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0) > gpurun_out/vggab_$n.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/vggab_$n.json'));print('vgg_hier $n', d['ms_per_step'])"
  done
done
