#!/bin/bash
# co-resident weight-gradient diagnosis: two identical backward passes with
# ASR_OVERLAP_WGRAD=2 (and =0 as control), per-layer dy / dx differences
set -o pipefail
mkdir -p gpurun_out
for mode in ${MODES:-2 0}; do
  echo "== mode $mode"
  DIAG_WHH=0.03 DIAG_H=${DIAG_H:-320} DIAG_L=${DIAG_L:-4} timeout -k 10 200 python -u -c "import sys; sys.argv=['x','trace','$mode']; sys.path.insert(0,'tools'); import buckets_diag as b; b.layer_trace()" > gpurun_out/cores_$mode.log 2>&1 || { tail -20 gpurun_out/cores_$mode.log; exit 1; }
  grep -v "^\[" gpurun_out/cores_$mode.log | grep -v Warning | tail -14
done
