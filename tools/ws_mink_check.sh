#!/bin/bash
# GPU box: short-K convs on the WS kernel (tuning conv_ws_mink 16 / 8 / 4)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ws_ab.py --key conv_ws_mink --arms 16,8,4 --set short_k --iters 20 --rounds 3 \
  > gpurun_out/mink_ab.log 2>&1 || { tail -20 gpurun_out/mink_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/mink_ab.log | tail -12
timeout -k 10 300 python -u tools/ab_inproc.py --switch tune:conv_ws_mink=8,16 --blocks 6 --steps 10 \
  > gpurun_out/mink_inproc.log 2>&1 || { tail -20 gpurun_out/mink_inproc.log; exit 1; }
tail -1 gpurun_out/mink_inproc.log
