#!/bin/bash
# Round-4 evidence on the GPU box: PMC traffic (eager step), the bench lines
# of every model path (training graphed + eager, inference x4), timed-region
# kernel profiles of the graphed training step, the per-shape conv table and
# the host-time split (graphed and eager).  Each GPU step has its own limit;
# the first failure ends the chain.
set -eo pipefail
tag=${1:-r4}
mkdir -p gpurun_out
bash tools/pmc_traffic.sh $tag --steps 3 --warmup 2
cp gpurun_out/${tag}_pmc.json profiles/${tag}_train_pmc.json
timeout -k 10 400 python3 bench.py > gpurun_out/${tag}_bench_train.log 2>&1

timeout -k 10 400 python3 bench.py --mask-fixed-rows --cpu-baseline 0 > gpurun_out/${tag}_bench_fixedrows.log 2>&1
timeout -k 10 400 python3 bench.py --mode infer > gpurun_out/${tag}_bench_infer.log 2>&1
timeout -k 10 400 python3 bench.py --model faster_rcnn_R_50_FPN --mode infer --cpu-baseline 0 > gpurun_out/${tag}_bench_c2.log 2>&1
timeout -k 10 400 python3 bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/${tag}_bench_retinanet.log 2>&1
timeout -k 10 400 python3 bench.py --model retinanet_R_101_FPN --mode train --cpu-baseline 0 > gpurun_out/${tag}_bench_retinanet_train.log 2>&1
timeout -k 10 400 python3 bench.py --model solo_v2_R_50_FPN --mode infer > gpurun_out/${tag}_bench_solo.log 2>&1
bash tools/profile_bench.sh ${tag}_train --steps 5 --warmup 3
timeout -k 10 300 python3 tools/conv_shapes.py > gpurun_out/${tag}_conv_shapes.txt 2>&1
timeout -k 10 300 python3 tools/host_time.py --steps 7 > gpurun_out/${tag}_host_time.log 2>&1
for m in train fixedrows infer c2 retinanet retinanet_train solo; do tail -1 gpurun_out/${tag}_bench_$m.log | cut -c1-300; done
tail -2 gpurun_out/${tag}_host_time.log
