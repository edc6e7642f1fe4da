#!/bin/bash
# round 5: which packed-FP32 operand selections are affected (single instructions)
set -o pipefail
mkdir -p gpurun_out
for P in 12 13 14 15 16; do
  timeout -k 10 60 tools/ubench/pk_hazard_$P 2 2 > gpurun_out/r05_pkh_$P.log 2>&1 || { echo "pattern $P rc=$?"; cat gpurun_out/r05_pkh_$P.log; exit 1; }
  grep -v "^pattern 0" gpurun_out/r05_pkh_$P.log
done
