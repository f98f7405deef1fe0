#!/bin/bash
# Ablation of the conv kernels (run on the GPU box): D2MI_CONV_DBG bits
# 1 = no global loads, 2 = no split / LDS writes, 4 = no MFMAs, for the old
# single-buffered kernel (arm 0) and the warp-specialised one (arm 3).
mkdir -p gpurun_out
S="2,200,336,256,256,3,1,plain;2,50,84,256,1024,1,1,r;2,100,168,128,128,3,1,plain"
for d in 0 1 2 3 4 5 6; do
  echo "== DBG=$d"
  D2MI_CONV_DBG=$d timeout -k 10 120 python -u tools/ws_ab.py --arms 0,3 --shapes "$S" --iters 10 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
done
