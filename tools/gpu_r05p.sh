#!/bin/bash
# round 5: LSE epilogue with DPP reductions, batched partial fold, f32 perm; CTC head kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_ctc_gpu.py -x -q --timeout 150 --timeout-method thread -m gpu > gpurun_out/p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/p_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_prof -- python3 tools/ctc_head_bench.py > gpurun_out/p_head.log 2>&1
rc=$?; grep "us / iteration" gpurun_out/p_head.log; [ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/p_prof -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
for x in sorted(r,key=lambda x:-float(x['TotalDurationNs']))[:14]: print('%-60s %6s %10.1f' % (x['Name'][:60], x['Calls'], float(x['AverageNs'])/1000))"
for v in "1:" "0:ASR_CTC_LSE_EPI=0"; do n=${v%%:*}; e=${v#*:}
env $e timeout -k 10 300 python -u bench.py --config vgg_hier --steps 10 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/p_vgg$n.json 2> gpurun_out/p_vgg$n.err || { tail -3 gpurun_out/p_vgg$n.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/p_vgg$n.json'));r=d['roofline']
print('vgg_hier bf16 epi=$n', d['ms_per_step'], [(k[:40], v.get('mean_launch_us')) for k,v in r.get('other_kernels',{}).items() if 'ctc' in k or 'gemm_bf16_8r<0, 0>' in k])"
done
timeout -k 10 300 python -u bench.py --config vgg_hier --precision fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/p_vgg32.json 2> gpurun_out/p_vgg32.err || { tail -3 gpurun_out/p_vgg32.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/p_vgg32.json'));r=d['roofline']
print('vgg_hier fp32', d['ms_per_step'], r['kernel'], r['mean_launch_us'], [(k[:40], v.get('mean_launch_us'), v.get('launches')) for k,v in r.get('other_kernels',{}).items()])"
