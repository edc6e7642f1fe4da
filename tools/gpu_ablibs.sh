#!/bin/bash
# same-box interleaved A/B of library builds (ASR_LIB_PATH), one bench config.
# usage: tools/gpu_ablibs.sh PFX CONFIG REPS name=path ...
PFX=$1; CFG=$2; REPS=$3; shift 3
mkdir -p gpurun_out
for i in $(seq $REPS); do
  for nv in "$@"; do
    n=${nv%%=*}; p=${nv#*=}
    ASR_LIB_PATH=$p timeout -k 10 200 python -u bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0 > gpurun_out/${PFX}_${n}_$i.json 2> gpurun_out/${PFX}_${n}_$i.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${PFX}_${n}_$i.json'));r=d['roofline'];o=r.get('other_kernels',{});print('$n', d['ms_per_step'], r.get('kernel'), r['mean_launch_us'], o.get('lstm_fwd_pass',{}).get('mean_launch_us'), o.get('gemm',{}).get('mean_launch_us'))"
  done
done
