#!/bin/bash
# round 5: f32 fast GEMM tiles + k tail, fp32 fused CTC head -- tests, GEMM rates, fp32 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_encoder_gpu.py tests/test_model_ctc.py tests/test_hierarchical.py tests/test_ctc_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/m_tests.log 2>&1
rc=$?; tail -5 gpurun_out/m_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_f32_bench.py > gpurun_out/m_f32g.log 2>&1
rc=$?; cat gpurun_out/m_f32g.log; [ $rc -eq 0 ] || exit $rc
for c in att4x320 vgg_hier; do
  timeout -k 10 300 python -u bench.py --config $c --precision fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/m_$c.json 2> gpurun_out/m_$c.err || { tail -3 gpurun_out/m_$c.err; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/m_$c.json'));r=d['roofline']
print('$c', d['ms_per_step'], r.get('kernel'), r['mean_launch_us'], r.get('share_of_timed_kernel_time'))
for k,v in r.get('other_kernels',{}).items(): print('   ', k[:40], v.get('mean_launch_us'), v.get('launches'), v.get('share_of_timed_kernel_time'))"
done
ASR_XG32_XU=16 timeout -k 10 300 python -u bench.py --config att4x320 --precision fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/m_att16.json 2> gpurun_out/m_att16.err || { tail -3 gpurun_out/m_att16.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/m_att16.json'));r=d['roofline']
print('att4x320 XU16', d['ms_per_step'], [(k[:20], v.get('mean_launch_us')) for k,v in r.get('other_kernels',{}).items() if 'lstm' in k], r['kernel'], r['mean_launch_us'])"
