#!/bin/bash
# SQ counters of the GEMM microbench (one pass per group)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -o "SQ_[A-Z_0-9]*" $OUT/counters.txt | sort -u | tr '\n' ' ' | head -c 3000; echo
rm -rf $OUT/pmc_g1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/pmc_g1 -- python3 $R/tools/gemm_bench.py > $OUT/pmc_g1.log 2>&1 || { tail -5 $OUT/pmc_g1.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections, os
R = os.environ.get('GRAFT_REPO_ROOT', '.')
f = glob.glob(R + '/gpurun_out/pmc_g1/**/*counter_collection.csv', recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'][:50]
    if 'gemm' not in k: continue
    agg[(k, r.get('Grid_Size', r.get('Grid_Size_X')))][r['Counter_Name']] += float(r['Counter_Value'])
for k, v in agg.items():
    print(k, {c: '%.3g' % x for c, x in v.items()})
PY
