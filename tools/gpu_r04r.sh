#!/bin/bash
# round 4: CTC lattice chunk preloads (single- and multi-wave) A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ctc_gpu.py tests/test_model_ctc.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/r04r_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r04r_tests.log; [ $rc = 0 ] || exit 1
for m in 0 1 0 1; do echo "== lattice_mw=$m"; ASR_CTC_LATTICE_MW=$m timeout -k 10 120 python -u tools/ctc_bench.py 2>&1 | grep -v amdgpu.ids | python3 -c "
import sys,json
for l in sys.stdin:
    try: d=json.loads(l)
    except Exception: print(l.strip()); continue
    print(d['kernel'], d['T'], d['V'], d['us_per_call'])" || exit 1; done
