#!/bin/bash
# Round-end evidence, part B (run on the GPU box): the inference / RetinaNet /
# SOLOv2 / Faster R-CNN / fixed-mask-rows bench lines, two timed-region
# profiles and the per-shape conv table.  usage: tools/refresh_b.sh <round tag>
set -eo pipefail
tag=$1
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --mode infer > gpurun_out/${tag}_bench_infer.log 2>&1
timeout -k 10 400 python3 bench.py --model faster_rcnn_R_50_FPN --mode infer > gpurun_out/${tag}_bench_c2.log 2>&1
timeout -k 10 400 python3 bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/${tag}_bench_retinanet.log 2>&1
timeout -k 10 400 python3 bench.py --model solo_v2_R_50_FPN --mode infer > gpurun_out/${tag}_bench_solo.log 2>&1
timeout -k 10 400 python3 bench.py --mask-fixed-rows --cpu-baseline 0 > gpurun_out/${tag}_bench_fixedrows.log 2>&1
bash tools/profile_bench.sh ${tag}_solo --model solo_v2_R_50_FPN --mode infer --steps 5 --warmup 3
bash tools/profile_bench.sh ${tag}_retinanet --model retinanet_R_101_FPN --mode infer --steps 5 --warmup 3
timeout -k 10 300 python3 tools/conv_shapes.py > gpurun_out/${tag}_conv_shapes.txt 2>&1
for m in infer c2 retinanet solo fixedrows; do tail -1 gpurun_out/${tag}_bench_$m.log | cut -c1-200; done
