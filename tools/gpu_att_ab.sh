#!/bin/bash
# attention decoder change: persistent-pass tests, then an interleaved A/B of the
# HEAD library (ab/libasr_hip_head.so) against the working tree on att4x320 / hybrid4x320
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_attdec_persist.py tests/test_attention_prod.py tests/test_parity_pins_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "att" > gpurun_out/att_ab_tests.log 2>&1; rc=$?
tail -4 gpurun_out/att_ab_tests.log
[ $rc -eq 0 ] || exit $rc
for C in ${CONFIGS:-hybrid4x320}; do
  for i in 1 2; do
    for nv in head=ab/old new=.; do
      n=${nv%%=*}; p=${nv#*=}
      (cd $p && timeout -k 10 200 python -u bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0) > gpurun_out/attab_${C}_$n.json 2>/dev/null || exit 1
      python -c "import json;d=json.load(open('gpurun_out/attab_${C}_$n.json'));o=d['roofline']['other_kernels'];print('$C $n', d['ms_per_step'], o.get('attdec_bwd_pass',{}).get('mean_launch_us'), o.get('attdec_fwd_pass',{}).get('mean_launch_us'))"
    done
  done
done
