#!/bin/bash
# round 5: f32 GEMM ring A/B, LSE epilogue + CTC forward from partials, generic-f32 list
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_ctc_gpu.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/o_tests.log 2>&1
rc=$?; tail -3 gpurun_out/o_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/gemm_f32_bench.py > gpurun_out/o_f32g2.log 2>&1 || exit 1
ASR_GEMM_F32_STAGES=3 timeout -k 10 300 python -u tools/gemm_f32_bench.py > gpurun_out/o_f32g3.log 2>&1 || exit 1
paste gpurun_out/o_f32g2.log gpurun_out/o_f32g3.log | cut -c1-160
for v in "1:" "0:ASR_CTC_LSE_EPI=0"; do n=${v%%:*}; e=${v#*:}
env $e timeout -k 10 300 python -u bench.py --config vgg_hier --steps 10 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/o_vgg$n.json 2> gpurun_out/o_vgg$n.err || { tail -3 gpurun_out/o_vgg$n.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/o_vgg$n.json'));r=d['roofline']
print('vgg_hier bf16 epi=$n', d['ms_per_step'], [(k[:40], v.get('mean_launch_us')) for k,v in r.get('other_kernels',{}).items() if 'ctc' in k or 'gemm_bf16_8r' in k])"
done
ASR_GEMM_DEBUG=1 timeout -k 10 300 python -u bench.py --config vgg_hier --precision fp32 --steps 1 --warmup 1 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/o_vgg32.json 2> gpurun_out/o_vgg32.err || { tail -3 gpurun_out/o_vgg32.err; exit 1; }
grep "generic f32" gpurun_out/o_vgg32.err | sort | uniq -c | head -20
