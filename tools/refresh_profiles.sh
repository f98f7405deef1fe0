#!/bin/bash
# Round-end evidence refresh (run on the GPU box): PMC traffic passes, the
# timed-region kernel profile, the default bench line (reads the fresh PMC
# file), the inference bench line and the per-shape conv table.
# usage: tools/refresh_profiles.sh <tag>
set -eo pipefail
tag=$1
mkdir -p gpurun_out
bash tools/pmc_traffic.sh $tag --steps 3 --warmup 2
cp gpurun_out/${tag}_pmc.json profiles/r1_train_pmc.json
timeout -k 10 400 python3 bench.py > gpurun_out/${tag}_bench_train.log 2>&1
timeout -k 10 400 python3 bench.py --mode infer > gpurun_out/${tag}_bench_infer.log 2>&1
bash tools/profile_bench.sh $tag --steps 5 --warmup 3
timeout -k 10 300 python3 tools/conv_shapes.py > gpurun_out/${tag}_conv_shapes.txt 2>&1
tail -1 gpurun_out/${tag}_bench_train.log
tail -1 gpurun_out/${tag}_bench_infer.log
