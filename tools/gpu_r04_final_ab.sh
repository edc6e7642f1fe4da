#!/bin/bash
# round-4 end: (a) whole GPU suite + smoke, then (b) the bench lines
set -o pipefail
bash tools/gpu_r04_final_a.sh || exit 1
bash tools/gpu_r04_final_b.sh || exit 1
