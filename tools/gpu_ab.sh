#!/bin/bash
# interleaved whole-step A/B of environment switches: VARIANTS="A=1 B=0;..." (';'-separated)
set -o pipefail
IFS=';' read -ra VS <<< "${VARIANTS}"
for r in 1 2; do
  for v in "${VS[@]}"; do
    # a variant may carry bench arguments after ' -- ' (e.g. "A=1 -- --sync-each-step")
    ev=${v%% -- *}; ba=""; [[ "$v" == *" -- "* ]] && ba=${v#* -- }
    out=$(env $ev timeout -k 10 200 python -u bench.py --config ${CONFIG:-ctc5x512} --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline $ba 2>&1 | tail -1)
    echo "[$v] $(echo $out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>/dev/null || echo $out | cut -c1-200)"
  done
done
