#!/bin/bash
# round 4: vectorised bf16 CTC gradient, saturated-gate pins, act_h encode/decode cost A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/ctc_bench.py > gpurun_out/r04_ctc_bench.jsonl 2>&1 || { tail -20 gpurun_out/r04_ctc_bench.jsonl; exit 1; }
grep V.:.10001 gpurun_out/r04_ctc_bench.jsonl | cut -c1-200
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_ctc_gpu.py tests/test_recurrence_full.py -s > gpurun_out/r04f_tests.log 2>&1
echo "tests rc=$?"; grep -E "saturated|passed|failed|Error" gpurun_out/r04f_tests.log | cut -c1-400 | tail -8
R=$(pwd)
for i in 1 2 3; do
  for v in enc plain; do
    if [ $v = plain ]; then L=$R/ablib/plain/libasr_hip.so; else L=$R/pytorch_end2end_speech_recognition_amd/libasr_hip.so; fi
    ASR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --config ctc5x512 --steps 15 --warmup 3 --no-cpu-baseline --h2d-steps 0 > gpurun_out/acth_${v}_$i.json 2> gpurun_out/acth_${v}_$i.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/acth_${v}_$i.json'));r=d['roofline'];o=r['other_kernels'];print('$v', d['ms_per_step'], r['kernel'], r['mean_launch_us'], o.get('lstm_fwd_xgx<*>',{}).get('mean_launch_us'))"
  done
done
