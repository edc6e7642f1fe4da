#!/bin/bash
# round 4: mode 3 vs mode 0 at the H = 320 configs (interleaved), then one default bench line each
set -o pipefail
for C in att4x320 hybrid4x320 timit2x320 vgg_hier; do
  echo "== $C"
  CONFIG=$C STEPS=15 VARIANTS="ASR_OVERLAP_WGRAD=0;ASR_OVERLAP_WGRAD=auto" timeout -k 10 500 bash tools/gpu_ab.sh || exit 1
done
