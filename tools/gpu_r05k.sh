#!/bin/bash
# round 5: f32 persistent recurrence -- unit tests, fp32 model goldens, fp32 bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_encoder_gpu.py -x -q --timeout 120 --timeout-method thread -m gpu -k "f32_persistent or golden or random_vs_oracle or backward_db or padded" > gpurun_out/k_enc.log 2>&1
rc=$?; tail -5 gpurun_out/k_enc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_parity_pins_gpu.py tests/test_attention_prod.py tests/test_model_ctc.py tests/test_hierarchical.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/k_models.log 2>&1
rc=$?; tail -5 gpurun_out/k_models.log; [ $rc -eq 0 ] || exit $rc
for c in att4x320 vgg_hier; do
  timeout -k 10 300 python -u bench.py --config $c --precision fp32 --steps 10 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/k_$c.json 2> gpurun_out/k_$c.err || { tail -3 gpurun_out/k_$c.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/k_$c.json'));r=d['roofline'];o=r.get('other_kernels',{});print('$c', d['ms_per_step'], r.get('kernel')[:40], r['mean_launch_us'], [(k[:30], v['mean_launch_us']) for k,v in o.items()][:8])"
done
