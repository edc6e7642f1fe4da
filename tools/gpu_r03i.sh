#!/bin/bash
# same-box interleaved A/B: 90c129f build (ab/old) vs HEAD (ACT_H 0/1), ctc5x512
mkdir -p gpurun_out
one() {  # tag dir env...
  local tag=$1 dir=$2; shift 2
  (cd $dir && env "$@" timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --h2d-steps 0) > gpurun_out/${PFX:-r03i}_$tag.json 2> gpurun_out/${PFX:-r03i}_$tag.err || return 1
  python -c "import json;d=json.load(open('gpurun_out/${PFX:-r03i}_$tag.json'));r=d['roofline'];print('$tag', d['ms_per_step'], r['mean_launch_us'], r['other_kernels']['lstm_fwd_pass']['mean_launch_us'], r['other_kernels']['gemm']['mean_launch_us'])"
}
for i in 1 2; do
  one old_$i ab/old && one new_$i . && one new0_$i . ASR_XG_ACT_H=0 || exit 1
done
