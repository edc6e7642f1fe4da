#!/bin/bash
# CTC kernels on the GPU: parity tests, the standalone fwd+bwd bench, and its
# rocprofv3 kernel-trace stats (gpurun_out/ctc_kstats.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ctc_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ctc_tests.log 2>&1 || { tail -30 gpurun_out/ctc_tests.log; exit 1; }
tail -2 gpurun_out/ctc_tests.log
timeout -k 10 120 python -u tools/ctc_bench.py > gpurun_out/ctc_bench.log 2>&1 || { tail -20 gpurun_out/ctc_bench.log; exit 1; }
cat gpurun_out/ctc_bench.log
cd /tmp && export TMPDIR=/tmp && rm -rf $R/gpurun_out/ktrace_ctc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ktrace_ctc -- python3 $R/tools/ctc_bench.py > $R/gpurun_out/ktrace_ctc.log 2>&1 || { tail -20 $R/gpurun_out/ktrace_ctc.log; exit 1; }
KT=$(find $R/gpurun_out/ktrace_ctc -name '*kernel_trace.csv' -print -quit)
python3 $R/profiles/kstats.py $KT > $R/gpurun_out/ctc_kstats.txt && head -20 $R/gpurun_out/ctc_kstats.txt
