#!/bin/bash
# GPU box: tuning conv_ws_levels in the inference paths that use the
# multi-level conv (Mask R-CNN RPN head, RetinaNet and SOLOv2 towers).
set -o pipefail
mkdir -p gpurun_out
for m in mask_rcnn_R_50_FPN retinanet_R_101_FPN solo_v2_R_50_FPN; do
  timeout -k 10 300 python -u tools/ab_inproc.py --mode infer --model $m --switch tune:conv_ws_levels \
    --blocks 8 --steps 10 > gpurun_out/wslv_infer_$m.log 2>&1 || { tail -20 gpurun_out/wslv_infer_$m.log; exit 1; }
  echo "$m: $(tail -1 gpurun_out/wslv_infer_$m.log)"
done
