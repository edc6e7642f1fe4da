#!/bin/bash
# round 5: packed-FP32 op_sel hazard probe, one binary per pattern, memory aggressor only
set -o pipefail
mkdir -p gpurun_out
for P in 4 7 8 9 11 10; do
  timeout -k 10 60 tools/ubench/pk_hazard_$P 2 2 > gpurun_out/r05_pkh_$P.log 2>&1 || { echo "pattern $P rc=$?"; cat gpurun_out/r05_pkh_$P.log; exit 1; }
  cat gpurun_out/r05_pkh_$P.log
done
