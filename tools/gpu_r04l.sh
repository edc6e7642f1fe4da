#!/bin/bash
# round 4: pipelined dX (opt-in) A/B across configs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_dx_pipeline_gpu.py > gpurun_out/r04l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04l_tests.log
[ $rc = 0 ] || exit 1
for c in ctc5x512 att4x320 vgg_hier timit2x320; do
  for v in 0 1; do
    ASR_DX_PIPE=$v timeout -k 10 200 python -u bench.py --config $c --steps 12 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/dxp_${c}_$v.json 2> gpurun_out/dxp_${c}_$v.err || { tail gpurun_out/dxp_${c}_$v.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/dxp_${c}_$v.json'));print('$c', '$v', d['ms_per_step'])"
  done
done
