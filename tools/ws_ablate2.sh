#!/bin/bash
# WS kernel ablation on mid-size shapes (run on the GPU box): D2MI_CONV_DBG
# 1 no loads, 2 no staging writes, 4 no MFMAs, 8 no epilogue; arm 2 = WS
S="2,50,84,1024,256,1,1,plain;2,50,84,256,256,3,1,plain;2,100,168,512,128,1,1,g;2,25,42,512,512,3,1,plain;2,200,336,256,256,3,1,plain"
for d in 0 3 4 7 8 15; do
  echo "== DBG=$d"
  D2MI_CONV_DBG=$d timeout -k 10 120 python -u tools/ws_ab.py --arms 0,2 --shapes "$S" --iters 10 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
done
