#!/bin/bash
# round 5: f32 fast GEMM -- exactness tests, fp32 GEMM throughput, fp32 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "f32_fast" > gpurun_out/l_gemm.log 2>&1
rc=$?; tail -5 gpurun_out/l_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_f32_bench.py > gpurun_out/l_f32g.log 2>&1
rc=$?; cat gpurun_out/l_f32g.log; [ $rc -eq 0 ] || exit $rc
ASR_GEMM_F32FAST=0 GEMM_BENCH_ONLY=lstm timeout -k 10 300 python -u tools/gemm_f32_bench.py > gpurun_out/l_f32g0.log 2>&1
rc=$?; cat gpurun_out/l_f32g0.log; [ $rc -eq 0 ] || exit $rc
for c in att4x320 vgg_hier; do
  timeout -k 10 300 python -u bench.py --config $c --precision fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/l_$c.json 2> gpurun_out/l_$c.err || { tail -3 gpurun_out/l_$c.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/l_$c.json'));r=d['roofline']
print('$c', d['ms_per_step'], r.get('kernel'), r['mean_launch_us'], r.get('share_of_timed_kernel_time'))
for k,v in r.get('other_kernels',{}).items(): print('   ', k[:40], v.get('mean_launch_us'), v.get('launches'), v.get('share_of_timed_kernel_time'))"
done
