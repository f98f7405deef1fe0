#!/bin/bash
# GPU box: the 16-deep multi-stage WS conv (tuning conv_ws = 4 / 5 / 6) against
# the 32-deep two-stage kernel (2): conv tests under D2MI_CONV_WS, per-shape
# A/B with bit-identity, in-step A/B.
set -o pipefail
mkdir -p gpurun_out
for v in ${WS_ARMS_TEST:-4}; do
  D2MI_CONV_WS=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_ops.py -k "conv" > gpurun_out/ws16_tests_$v.log 2>&1 || { tail -30 gpurun_out/ws16_tests_$v.log; exit 1; }
  tail -1 gpurun_out/ws16_tests_$v.log
done
timeout -k 10 400 python -u tools/ws_ab.py --key conv_ws --arms ${WS_ARMS:-2,4,5,6} --set kxk,short_k --iters 20 --rounds 3 \
  > gpurun_out/ws16_ab.log 2>&1 || { tail -20 gpurun_out/ws16_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ws16_ab.log | tail -20
timeout -k 10 300 python -u tools/ab_inproc.py --switch tune:conv_ws=${WS_ON:-4},2 --blocks 6 --steps 10 \
  > gpurun_out/ws16_inproc.log 2>&1 || { tail -20 gpurun_out/ws16_inproc.log; exit 1; }
tail -1 gpurun_out/ws16_inproc.log
timeout -k 10 400 python -u tools/ws_ab.py --key conv_xcd --arms 0,1 --set kxk,short_k --iters 20 --rounds 3 \
  > gpurun_out/conv_xcd_ab.log 2>&1 || { tail -20 gpurun_out/conv_xcd_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/conv_xcd_ab.log | tail -1
timeout -k 10 300 python -u tools/ab_inproc.py --switch tune:conv_xcd --blocks 6 --steps 10 \
  > gpurun_out/conv_xcd_inproc.log 2>&1 || { tail -20 gpurun_out/conv_xcd_inproc.log; exit 1; }
tail -1 gpurun_out/conv_xcd_inproc.log
