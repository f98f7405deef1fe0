#!/bin/bash
# GPU box: weight planes (d2mi_conv2d_nhwc_w3) -- parity tests, per-shape A/B of
# the kernels that take them (tuning conv_bp 0 vs 7), in-step A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_planes.py tests/test_gpu_ops.py -k "planes or conv" > gpurun_out/planes_tests.log 2>&1 \
  || { tail -40 gpurun_out/planes_tests.log; exit 1; }
tail -1 gpurun_out/planes_tests.log
timeout -k 10 400 python -u tools/ws_ab.py --key conv_bp --arms 0,7,1 --planes --set kxk,short_k --iters 20 --rounds 3 \
  > gpurun_out/planes_ab.log 2>&1 || { tail -20 gpurun_out/planes_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/planes_ab.log | tail -18
timeout -k 10 300 python -u tools/ab_inproc.py --switch weight_planes --blocks 6 --steps 10 \
  > gpurun_out/planes_inproc.log 2>&1 || { tail -20 gpurun_out/planes_inproc.log; exit 1; }
tail -1 gpurun_out/planes_inproc.log
