#!/bin/bash
# (1) co-residency diagnostics: no split-K slabs; (2) vgg_hier A/B of the fast
# kernel's / 256x64 kernel's LDS stages; (3) exact conv GEMM tests; (4) GEMM PMC
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u tools/buckets_diag.py trace 2 2>&1 | grep -v amdgpu.ids > gpurun_out/r03f_$name.log; local rc=$?
  echo "== $name rc=$rc"; grep "dx\|diag" gpurun_out/r03f_$name.log
  return $rc
}
run nosplit DIAG_WHH=0.03 ASR_GEMM_NOSPLIT=1 && run nosplit_b DIAG_WHH=0.03 ASR_GEMM_NOSPLIT=1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_vgg.py -m gpu -q -k tap_gemm --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03f_tap.log 2>&1; rc=$?
echo "tap tests rc=$rc"; tail -3 gpurun_out/r03f_tap.log
if [ $rc -ne 0 ]; then exit 1; fi
for i in 1 2; do
  for v in "2 2" "4 2" "2 3" "4 3"; do
    set -- $v
    ASR_GEMM_STAGES=$1 ASR_GEMM_N64_STAGES=$2 timeout -k 10 200 python -u bench.py --config vgg_hier --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0 > gpurun_out/r03f_vgg.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r03f_vgg.json'));print('STAGES=$1 N64=$2', d['ms_per_step'])"
  done
done
bash tools/gemm_pmc_r03.sh
