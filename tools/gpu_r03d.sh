#!/bin/bash
# (1) two-bit tag determinism experiment, (2) recurrence tests with packed fp16
# activations, (3) interleaved A/B of ctc5x512 with ASR_XG_ACT_H=0/1
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u tools/buckets_diag.py trace 2 2>&1 | grep -v amdgpu.ids > gpurun_out/r03d_$name.log; local rc=$?
  echo "== $name rc=$rc"; grep "dx" gpurun_out/r03d_$name.log
  return $rc
}
run tag2 ASR_XG_TAG2=1 && run tag2b ASR_XG_TAG2=1 && run tag1 ASR_XG_TAG2=0 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_recurrence_full.py tests/test_encoder_gpu.py tests/test_model_ctc.py -m gpu -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|max err" gpurun_out/r03d_tests.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  for a in 0 1; do
    ASR_XG_ACT_H=$a timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0 > gpurun_out/r03d_ab_$a.json 2>gpurun_out/r03d_ab_$a.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r03d_ab_$a.json'));r=d['roofline'];print('ACT_H=$a', d['ms_per_step'], r['mean_launch_us'], r['other_kernels']['lstm_fwd_pass']['mean_launch_us'])"
  done
done
timeout -k 10 200 python -u bench.py --config hybrid4x320 --steps 10 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/r03d_hybrid.json 2>gpurun_out/r03d_hybrid.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r03d_hybrid.json'));r=d['roofline'];print(d['ms_per_step'], json.dumps({k:v for k,v in r['other_kernels'].items() if k.startswith('att')}))"
