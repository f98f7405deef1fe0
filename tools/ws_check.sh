#!/bin/bash
# WS conv A/B + ablation (run on the GPU box)
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ws_ab.py --arms 0,2 --set kxk,short_k --iters 20 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
S="2,200,336,256,256,3,1,plain;2,100,168,128,128,3,1,plain;2,50,84,256,1024,1,1,r"
for d in 3 4; do
  echo "== DBG=$d"
  D2MI_CONV_DBG=$d timeout -k 10 120 python -u tools/ws_ab.py --arms 0,2 --shapes "$S" --iters 10 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
done
