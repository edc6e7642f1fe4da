#!/bin/bash
# round-5 end (b): bench lines of the five configs (bf16, with cpu_baseline and
# parity) and fp32-mode lines of the configs BASELINE quotes without bf16
set -o pipefail
mkdir -p gpurun_out
for c in ctc5x512 timit2x320 att4x320 hybrid4x320 vgg_hier; do
  timeout -k 10 400 python -u bench.py --config $c > gpurun_out/r05_bench_$c.json 2> gpurun_out/r05_bench_$c.err || { tail gpurun_out/r05_bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05_bench_$c.json'));print('$c', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'])"
done
for c in vgg_hier att4x320 hybrid4x320; do
  timeout -k 10 300 python -u bench.py --config $c --precision fp32 --no-cpu-baseline --no-parity > gpurun_out/r05_bench_${c}_fp32.json 2> gpurun_out/r05_bench_${c}_fp32.err || { tail gpurun_out/r05_bench_${c}_fp32.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05_bench_${c}_fp32.json'));print('$c fp32', d['ms_per_step'])"
done
