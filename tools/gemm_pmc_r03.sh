#!/bin/bash
# PMC passes of the 8-wave ring GEMM at each 5x512 shape (one rocprofv3 run per
# shape and counter group; kernel-trace only, no sys/runtime traces).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/gemm_pmc; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for S in fwd dX dW dWhh; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1)); rm -rf $OUT/${S}_$i
    GEMM_BENCH_ONLY="$S " timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/${S}_$i -- python3 $R/tools/gemm_bench.py > $OUT/${S}_$i.log 2>&1 || { echo "pmc $S $i failed"; tail -5 $OUT/${S}_$i.log; exit 1; }
  done
  echo "=== $S"; grep TF/s $OUT/${S}_1.log
  for j in 1 2 3 4; do python3 $R/tools/pmc_kernel.py $OUT/${S}_$j gemm_bf16 splitk; done
done
