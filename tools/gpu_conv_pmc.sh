#!/bin/bash
# PMC passes over the tap-resident conv kernels (one counter set per run)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/convpmc
cd /tmp && export TMPDIR=/tmp
export CONV_BENCH_ONLY_TR=1
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/convpmc/p$i -- python3 $R/tools/conv_bench.py > $R/gpurun_out/convpmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/convpmc/p$i.log; exit 1; }
done
python3 $R/tools/pmc_kernel.py $R/gpurun_out/convpmc conv3x3_tr 2>&1 | tail -40
