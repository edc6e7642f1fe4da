#!/bin/bash
# A/B of the VGG BN-moments pass shapes (ASR_VGG_BNM=<NT>x<U>) on vgg_hier
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 256x1 256x2 256x4 512x1 512x2 1024x1 1024x2; do
  rm -rf gpurun_out/bnm_$v
  ASR_VGG_BNM=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bnm_$v -- python3 bench.py --config vgg_hier --steps 4 --warmup 2 --no-cpu-baseline --no-parity > gpurun_out/bnm_$v.log 2>&1 || { echo "fail $v"; tail -5 gpurun_out/bnm_$v.log; exit 1; }
  f=$(find gpurun_out/bnm_$v -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv, json
r=list(csv.DictReader(open('$f')))
x=[q for q in r if 'bn_moments' in q['Name']]
ms=json.loads(open('gpurun_out/bnm_$v.log').read().strip().splitlines()[-1])['ms_per_step']
print('$v', ms, ['%s %s x%s' % (q['Name'][:40], round(float(q['AverageNs'])/1000,1), q['Calls']) for q in x])"
done
