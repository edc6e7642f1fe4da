#!/bin/bash
# same-box interleaved A/B of library builds over several configs (ASR_LIB_PATH).
# usage: tools/gpu_abcfg.sh PFX REPS "cfg1 cfg2" name=path ...
PFX=$1; REPS=$2; CFGS=$3; shift 3
mkdir -p gpurun_out
for i in $(seq $REPS); do
  for cfg in $CFGS; do
    for nv in "$@"; do
      n=${nv%%=*}; p=${nv#*=}
      ASR_LIB_PATH=$p timeout -k 10 240 python -u bench.py --config $cfg --steps 15 --warmup 3 --no-cpu-baseline --no-parity --h2d-steps 0 > gpurun_out/${PFX}_${cfg}_${n}_$i.json 2> gpurun_out/${PFX}_${cfg}_${n}_$i.err || { echo "FAILED $cfg $n"; tail -5 gpurun_out/${PFX}_${cfg}_${n}_$i.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/${PFX}_${cfg}_${n}_$i.json'));print('$cfg', '$n', d['ms_per_step'])"
    done
  done
done
