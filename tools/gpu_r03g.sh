#!/bin/bash
# vgg / conv tests with the bf16 conv output, then A/B of GEMM stages, then diag + PMC
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vgg.py tests/test_parity_pins_gpu.py tests/test_gemm_gpu.py -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03g_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed|vs float64" gpurun_out/r03g_tests.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
for i in 1 2; do
  for v in "2 2 1" "2 2 0" "4 2 1" "2 3 1"; do
    set -- $v
    ASR_GEMM_STAGES=$1 ASR_GEMM_N64_STAGES=$2 ASR_VGG_Z_BF16=$3 timeout -k 10 200 python -u bench.py --config vgg_hier --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0 > gpurun_out/r03g_vgg.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r03g_vgg.json'));print('STAGES=$1 N64=$2 ZBF=$3', d['ms_per_step'])"
  done
done
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u tools/buckets_diag.py trace 2 2>&1 | grep -v amdgpu.ids > gpurun_out/r03g_$name.log; local rc=$?
  echo "== $name rc=$rc"; grep "dx\|diag" gpurun_out/r03g_$name.log
  return $rc
}
run nosplit DIAG_WHH=0.03 ASR_GEMM_NOSPLIT=1 && run nosplit_b DIAG_WHH=0.03 ASR_GEMM_NOSPLIT=1 || exit 1
bash tools/gemm_pmc_r03.sh
