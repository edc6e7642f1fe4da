#!/bin/bash
# VALU vs memory for the VGG row passes: SQ counters on vgg_hier (one pass)
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc_rw -- python3 $R/bench.py --config vgg_hier --steps 3 --warmup 1 --no-cpu-baseline --no-parity --h2d-steps 0 > $R/gpurun_out/pmc_rw.log 2>&1 || { tail -5 $R/gpurun_out/pmc_rw.log; exit 1; }
python3 $R/tools/pmc_kernel.py $R/gpurun_out/pmc_rw rw_ conv3x3_c1 | cut -c1-250
