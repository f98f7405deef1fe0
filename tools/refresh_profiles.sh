#!/bin/bash
# Round-end evidence refresh (run on the GPU box): PMC traffic passes, the
# bench lines of every model path (the training line reads the fresh PMC
# file), timed-region kernel profiles and the per-shape conv table.
# usage: tools/refresh_profiles.sh <round tag, e.g. r2>
set -eo pipefail
tag=$1
mkdir -p gpurun_out
bash tools/pmc_traffic.sh $tag --steps 3 --warmup 2
cp gpurun_out/${tag}_pmc.json profiles/${tag}_train_pmc.json
timeout -k 10 400 python3 bench.py > gpurun_out/${tag}_bench_train.log 2>&1
timeout -k 10 400 python3 bench.py --mode infer > gpurun_out/${tag}_bench_infer.log 2>&1
timeout -k 10 400 python3 bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/${tag}_bench_retinanet.log 2>&1
timeout -k 10 400 python3 bench.py --model solo_v2_R_50_FPN --mode infer > gpurun_out/${tag}_bench_solo.log 2>&1
bash tools/profile_bench.sh ${tag}_train --steps 5 --warmup 3
bash tools/profile_bench.sh ${tag}_solo --model solo_v2_R_50_FPN --mode infer --steps 5 --warmup 3
bash tools/profile_bench.sh ${tag}_retinanet --model retinanet_R_101_FPN --mode infer --steps 5 --warmup 3
timeout -k 10 300 python3 tools/conv_shapes.py > gpurun_out/${tag}_conv_shapes.txt 2>&1
for m in train infer retinanet solo; do tail -1 gpurun_out/${tag}_bench_$m.log; done
