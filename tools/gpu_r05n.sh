#!/bin/bash
# round 5: f32 GEMM ring A/B, generic-f32 products of vgg_hier
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k f32 > gpurun_out/n_tests.log 2>&1
rc=$?; tail -3 gpurun_out/n_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_f32_bench.py > gpurun_out/n_f32g2.log 2>&1 || exit 1
ASR_GEMM_F32_STAGES=3 timeout -k 10 300 python -u tools/gemm_f32_bench.py > gpurun_out/n_f32g3.log 2>&1 || exit 1
paste gpurun_out/n_f32g2.log gpurun_out/n_f32g3.log | cut -c1-160
ASR_GEMM_DEBUG=1 timeout -k 10 300 python -u bench.py --config vgg_hier --precision fp32 --steps 1 --warmup 1 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/n_vgg.json 2> gpurun_out/n_vgg.err || { tail -3 gpurun_out/n_vgg.err; exit 1; }
grep "generic f32" gpurun_out/n_vgg.err | sort | uniq -c | head -20
