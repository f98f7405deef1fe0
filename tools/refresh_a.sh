#!/bin/bash
# Round-end evidence, part A (run on the GPU box): PMC traffic passes of the
# training bench, then the training bench line (reads the fresh PMC file) and
# its timed-region kernel profile.  usage: tools/refresh_a.sh <round tag>
set -eo pipefail
tag=$1
mkdir -p gpurun_out
bash tools/pmc_traffic.sh $tag --steps 3 --warmup 2
cp gpurun_out/${tag}_pmc.json profiles/${tag}_train_pmc.json
timeout -k 10 400 python3 bench.py > gpurun_out/${tag}_bench_train.log 2>&1
bash tools/profile_bench.sh ${tag}_train --steps 5 --warmup 3
tail -1 gpurun_out/${tag}_bench_train.log | cut -c1-300
