#!/bin/bash
# 1x1 weight-gradient split policy sweep (D2MI_WGRAD_MINCH / _SLOTS /
# _MAXSPLIT are read once per process: one process per setting), the
# training step's 1x1 wgrad shapes; per-shape medians and total per setting.
set -o pipefail
SH="2,50,84,1024,256,1,1,w;2,50,84,256,1024,1,1,w;2,100,168,128,512,1,1,w;2,100,168,512,128,1,1,w;2,200,336,256,256,1,1,w;2,200,336,64,256,1,1,w;2,200,336,256,64,1,1,w;2,100,168,256,512,1,1,w"
for cfg in "16 0 64" "16 0 128" "16 0 256" "8 768 256" "16 1024 256"; do
  set -- $cfg
  echo "== MINCH=$1 SLOTS=$2 MAXSPLIT=$3"
  D2MI_WGRAD_MINCH=$1 D2MI_WGRAD_SLOTS=$2 D2MI_WGRAD_MAXSPLIT=$3 timeout -k 10 200 python -u tools/ws_ab.py \
    --key wgrad_ws --arms 0 --iters 20 --rounds 3 --shapes "$SH" 2>&1 | grep -v amdgpu.ids || exit 1
done
