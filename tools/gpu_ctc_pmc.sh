#!/bin/bash
# HBM traffic of the CTC kernels at the ctc_bench shapes: one rocprofv3 --pmc
# pass per counter (FETCH_SIZE, WRITE_SIZE; no tracing beside --pmc), then the
# per-kernel means (tools/pmc_kernel.py).  gfx950 correction as in
# tools/pmc_traffic.py: bytes = 2 * FETCH_SIZE + WRITE_SIZE (KB units -> x1024).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT && cd /tmp && export TMPDIR=/tmp
rm -rf $OUT/ctc_pmc_fetch $OUT/ctc_pmc_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/ctc_pmc_fetch -- python3 $R/tools/ctc_bench.py > $OUT/ctc_pmc_fetch.log 2>&1 || { tail -20 $OUT/ctc_pmc_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/ctc_pmc_write -- python3 $R/tools/ctc_bench.py > $OUT/ctc_pmc_write.log 2>&1 || { tail -20 $OUT/ctc_pmc_write.log; exit 1; }
python3 $R/tools/pmc_kernel.py $OUT/ctc_pmc_fetch ctc_ > $OUT/ctc_pmc.txt && python3 $R/tools/pmc_kernel.py $OUT/ctc_pmc_write ctc_ >> $OUT/ctc_pmc.txt && cat $OUT/ctc_pmc.txt
