#!/bin/bash
# wgrad_ws1 (the WS weight-gradient kernel on 1x1 convs) on the GPU box:
# wgrad tests, per-shape A/B, in-step A/B.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "wgrad" 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 10 300 python -u tools/ws_ab.py --key wgrad_ws1 --arms 0,6 --iters 20 --rounds 3 \
  --shapes "2,50,84,1024,256,1,1,w;2,50,84,256,1024,1,1,w;2,100,168,512,128,1,1,w;2,200,336,256,256,1,1,w;2,100,168,256,512,1,1,w;2,200,336,256,512,1,2,w;2,100,168,512,1024,1,2,w;2,50,84,1024,2048,1,2,w" \
  2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u tools/ab_inproc.py --switch wgrad_ws1 --blocks 8 --steps 10 2>&1 | grep -v amdgpu.ids | tail -2
timeout -k 10 300 python -u tools/torch_prof.py --mode train --steps 3 --rows 150 --stacks > gpurun_out/torch_prof_stdout.txt 2>&1 || exit 1
