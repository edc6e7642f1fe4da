#!/bin/bash
# round 4: GEMM 8r k-loop unrolled by two (no B-fragment copies) A/B
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py > gpurun_out/r04p_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r04p_tests.log
[ $rc = 0 ] || exit 1
for i in 1 2; do
  for v in head cur; do
    if [ $v = head ]; then L=$R/ablib/head/libasr_hip.so; else L=$R/pytorch_end2end_speech_recognition_amd/libasr_hip.so; fi
    echo "== $v"; ASR_LIB_PATH=$L timeout -k 10 200 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
