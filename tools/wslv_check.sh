#!/bin/bash
# GPU box: the warp-specialised multi-level conv (tuning conv_ws_levels):
# its level tests, the RPN levels training test, the in-step A/B of the RPN
# head levels form on it vs per level, and the inference A/B (RetinaNet towers).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "conv_levels" > gpurun_out/wslv_tests.log 2>&1 || { grep -E "Error|error|assert|FAILED" gpurun_out/wslv_tests.log | head -30; tail -20 gpurun_out/wslv_tests.log; exit 1; }
tail -1 gpurun_out/wslv_tests.log
timeout -k 10 300 python -u tools/ab_inproc.py --switch rpn_levels_ws --blocks 8 --steps 10 \
  > gpurun_out/wslv_inproc.log 2>&1 || { tail -20 gpurun_out/wslv_inproc.log; exit 1; }
tail -1 gpurun_out/wslv_inproc.log
