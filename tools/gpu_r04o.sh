#!/bin/bash
# round 4: VGG row walk A/B (ablib/head = per-row loops)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_vgg_rows_gpu.py tests/test_parity_pins_gpu.py > gpurun_out/r04o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04o_tests.log
[ $rc = 0 ] || exit 1
for i in 1 2; do
  for v in head cur; do
    if [ $v = head ]; then L=$R/ablib/head/libasr_hip.so; else L=$R/pytorch_end2end_speech_recognition_amd/libasr_hip.so; fi
    ASR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --config vgg_hier --steps 12 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/vw_${v}_$i.json 2> gpurun_out/vw_${v}_$i.err || { tail gpurun_out/vw_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/vw_${v}_$i.json'));print('$v', d['ms_per_step'])"
  done
done
bash tools/gpu_ktrace.sh vgg_hier r04rows > /dev/null && grep -E "rw_" gpurun_out/r04rows_kernel_stats_vgg_hier.txt | cut -c1-60,90-140
