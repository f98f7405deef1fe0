#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
STEPS=5 bash tools/profile_bench.sh r4aa_solo_train --model solo_v2_R_50_FPN --mode train --steps 5 --warmup 2
head -c 0 /dev/null
