#!/bin/bash
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python -u tools/buckets_diag.py trace 2 2>&1 | grep -v amdgpu.ids > gpurun_out/r03c_$name.log; local rc=$?
  echo "== $name rc=$rc"; grep "dx" gpurun_out/r03c_$name.log
  return $rc
}
run tag2 ASR_XG_TAG2=1 && run tag2b ASR_XG_TAG2=1 && run tag1 ASR_XG_TAG2=0
