#!/bin/bash
# GPU box: the in-launch split-K fix-up (tuning conv_fix): conv tests, the
# per-shape A/B (bit-identity across arms checked by ws_ab.py), the whole
# -m gpu suite, the in-step A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "conv" > gpurun_out/fix_conv_tests.log 2>&1 || { tail -30 gpurun_out/fix_conv_tests.log; exit 1; }
tail -1 gpurun_out/fix_conv_tests.log
timeout -k 10 400 python -u tools/ws_ab.py --key conv_fix --arms 0,1 --iters 20 --rounds 3 \
  > gpurun_out/fix_ab.log 2>&1 || { tail -20 gpurun_out/fix_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fix_ab.log | tail -40
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_fix.log 2>&1
rc=$?
tail -1 gpurun_out/gpu_tests_fix.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests_fix.log | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_inproc.py --switch tune:conv_fix=1,0 --blocks 8 --steps 10 \
  > gpurun_out/fix_inproc.log 2>&1 || { tail -20 gpurun_out/fix_inproc.log; exit 1; }
tail -1 gpurun_out/fix_inproc.log
