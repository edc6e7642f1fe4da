#!/bin/bash
# same-box interleaved A/B of bench.py between ab/prev (a worktree of an earlier
# commit, built in place) and this tree.  usage: tools/gpu_abtree.sh PFX CONFIG REPS [ENV...]
PFX=$1; CFG=$2; REPS=$3; shift 3
mkdir -p gpurun_out
one() {  # tag dir env...
  local tag=$1 dir=$2; shift 2
  (cd $dir && env "$@" timeout -k 10 200 python -u bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0) > gpurun_out/${PFX}_$tag.json 2> gpurun_out/${PFX}_$tag.err || return 1
  python -c "import json;d=json.load(open('gpurun_out/${PFX}_$tag.json'));r=d['roofline'];o=r.get('other_kernels',{});print('$tag', d['ms_per_step'], r.get('kernel'), r['mean_launch_us'], o.get('lstm_fwd_pass',{}).get('mean_launch_us'), o.get('gemm',{}).get('mean_launch_us'))"
}
for i in $(seq $REPS); do
  one prev_$i ab/prev "$@" && one new_$i . "$@" || exit 1
done
