#!/bin/bash
# Round-5 evidence on the GPU box, part A (train) or B (the other paths):
#   A: PMC traffic passes of the training bench, the training bench line (with
#      the CPU baseline and the fixed-rows object), the timed-region kernel profile;
#   B: inference lines (Mask R-CNN, Faster R-CNN C2, RetinaNet R101 C4, SOLOv2
#      C5), the RetinaNet training line, the per-shape conv table, host time.
# Each GPU step has its own limit; the first failure ends the chain.
set -eo pipefail
part=${1:-A}
tag=${TAG:-r5}
mkdir -p gpurun_out
if [ "$part" = A ]; then
  bash tools/pmc_traffic.sh $tag --steps 3 --warmup 2
  cp gpurun_out/${tag}_pmc.json profiles/${tag}_train_pmc.json
  timeout -k 10 500 python3 bench.py > gpurun_out/${tag}_bench_train.log 2>&1
  bash tools/profile_bench.sh ${tag}_train --steps 5 --warmup 3
  tail -1 gpurun_out/${tag}_bench_train.log | cut -c1-300
else
  timeout -k 10 400 python3 bench.py --mode infer > gpurun_out/${tag}_bench_infer.log 2>&1
  timeout -k 10 400 python3 bench.py --model faster_rcnn_R_50_FPN --mode infer --cpu-baseline 0 > gpurun_out/${tag}_bench_c2.log 2>&1
  timeout -k 10 400 python3 bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/${tag}_bench_retinanet.log 2>&1
  timeout -k 10 400 python3 bench.py --model retinanet_R_101_FPN --mode train --cpu-baseline 0 > gpurun_out/${tag}_bench_retinanet_train.log 2>&1
  timeout -k 10 400 python3 bench.py --model solo_v2_R_50_FPN --mode infer > gpurun_out/${tag}_bench_solo.log 2>&1
  timeout -k 10 300 python3 tools/conv_shapes.py > gpurun_out/${tag}_conv_shapes.txt 2>&1
  timeout -k 10 300 python3 tools/host_time.py --steps 7 > gpurun_out/${tag}_host_time.log 2>&1
  for m in infer c2 retinanet retinanet_train solo; do tail -1 gpurun_out/${tag}_bench_$m.log | cut -c1-300; done
  tail -1 gpurun_out/${tag}_host_time.log
fi
