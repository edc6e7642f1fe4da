#!/bin/bash
# SQ counters of the 8-wave GEMM at the 5x512 shapes (library off), one pass per group
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export ASR_GEMM_LIB=0
rm -rf $OUT/pmc8_1 $OUT/pmc8_2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/pmc8_1 -- python3 $R/tools/gemm_bench.py > $OUT/pmc8_1.log 2>&1 || { tail -5 $OUT/pmc8_1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU --output-format csv -d $OUT/pmc8_2 -- python3 $R/tools/gemm_bench.py > $OUT/pmc8_2.log 2>&1 || { tail -5 $OUT/pmc8_2.log; exit 1; }
python3 $R/tools/pmc_kernel.py $OUT/pmc8_1 gemm_bf16_8w
python3 $R/tools/pmc_kernel.py $OUT/pmc8_2 gemm_bf16_8w
