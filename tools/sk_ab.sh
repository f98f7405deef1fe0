#!/bin/bash
# conv_sk (stream-K WS conv) on the GPU box: conv parity tests, per-shape A/B
# (outputs compared, not bit-equal: different K split points), in-step A/B.
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "conv or linear or wgrad or stream" 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 10 300 python -u tools/ws_ab.py --key conv_sk --arms 0,1 --iters 20 --rounds 3 \
  --shapes "2,100,168,128,128,3,1,plain;2,100,168,128,128,3,1,g;2,50,84,1024,512,1,1,plain;2,100,168,512,128,1,1,g;2,50,84,256,256,3,1,plain" \
  2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u tools/ab_inproc.py --switch conv_sk --blocks 8 --steps 10 2>&1 | grep -v amdgpu.ids | tail -2
