#!/bin/bash
# 8-wave GEMM swizzle fix: exactness tests, throughput, conflicts, ctc5x512 step
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_recurrence_full.py tests/test_model_ctc.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03h_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r03h_tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/r03h_tests.log | head; exit 1; fi
timeout -k 10 120 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/gemm_pmc2; mkdir -p $OUT
for S in fwd dX; do
  GEMM_BENCH_ONLY="$S " timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $OUT/$S -- python3 $R/tools/gemm_bench.py > $OUT/$S.log 2>&1 || exit 1
  python3 $R/tools/pmc_kernel.py $OUT/$S gemm_bf16_8r
done
cd $R
for c in ctc5x512 att4x320; do
  timeout -k 10 200 python -u bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0 > gpurun_out/r03h_$c.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r03h_$c.json'));r=d['roofline'];print('$c', d['ms_per_step'], r['mean_launch_us'], r['other_kernels'].get('gemm'))"
done
