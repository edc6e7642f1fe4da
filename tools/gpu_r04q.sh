#!/bin/bash
# round 4: GEMM loop (unroll, dense K staging) + VGG walkers vs ablib/head
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
[ -n "$SKIP_TESTS" ] || { timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r04q_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/r04q_tests.log | tail -5
[ $rc = 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04q_smoke.log 2>&1 || { tail -5 gpurun_out/r04q_smoke.log; exit 1; }
tail -2 gpurun_out/r04q_smoke.log; }
for v in head cur; do
  if [ $v = head ]; then L=$R/ablib/head/libasr_hip.so; export ASR_VGG_C1_RELU_P=0; else unset ASR_VGG_C1_RELU_P; L=$R/pytorch_end2end_speech_recognition_amd/libasr_hip.so; fi
  echo "== $v"; ASR_LIB_PATH=$L timeout -k 10 200 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | grep TF || exit 1
done
for m in 0 1; do echo "== lattice_mw=$m"; ASR_CTC_LATTICE_MW=$m timeout -k 10 120 python -u tools/ctc_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done
timeout -k 10 120 python -u tools/blas_probe.py 2>&1 | grep TF || exit 1
for i in 1 2; do
  for c in vgg_hier ctc5x512; do
    for v in head cur; do
      if [ $v = head ]; then L=$R/ablib/head/libasr_hip.so; export ASR_VGG_C1_RELU_P=0; else unset ASR_VGG_C1_RELU_P; L=$R/pytorch_end2end_speech_recognition_amd/libasr_hip.so; fi
      ASR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --config $c --steps 12 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/q_${c}_${v}_$i.json 2> gpurun_out/q_${c}_${v}_$i.err || { tail gpurun_out/q_${c}_${v}_$i.err; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/q_${c}_${v}_$i.json'));r=d['roofline'];o=r['other_kernels'];print('$c $v', d['ms_per_step'], r['kernel'], r['mean_launch_us'], {k:v.get('mean_launch_us') for k,v in o.items() if 'lstm' in k})"
    done
  done
done
