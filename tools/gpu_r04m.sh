#!/bin/bash
# round 4 (mid): kernel stats of vgg_hier / hybrid4x320 for the next targets
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in vgg_hier hybrid4x320; do bash tools/gpu_ktrace.sh $C r04mid || exit 1; done
