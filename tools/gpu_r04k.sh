#!/bin/bash
# round 4: pipelined dX between stacked BLSTM layers
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_dx_pipeline_gpu.py tests/test_model_ctc.py -s > gpurun_out/r04k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "pipelined|FAIL|Error|passed|failed" gpurun_out/r04k_tests.log | cut -c1-400 | tail -14
[ $rc = 0 ] || exit 1
for i in 1 2; do
  for v in 0 1; do
    ASR_DX_PIPE=$v timeout -k 10 200 python -u bench.py --config ctc5x512 --steps 15 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/dxp_${v}_$i.json 2> gpurun_out/dxp_${v}_$i.err || { tail gpurun_out/dxp_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/dxp_${v}_$i.json'));r=d['roofline'];o=r['other_kernels'];print('$v', d['ms_per_step'], r['kernel'], r['mean_launch_us'], {k:v.get('mean_launch_us') for k,v in o.items() if 'lstm' in k})"
  done
done
ASR_DX_PIPE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_pipe -o kt -- python3 bench.py --config ctc5x512 --steps 3 --warmup 2 --no-cpu-baseline --h2d-steps 0 > gpurun_out/kt_pipe.log 2>&1 || { tail -5 gpurun_out/kt_pipe.log; exit 1; }
find gpurun_out/kt_pipe -name "*.csv" | head
