#!/bin/bash
# GPU box: conv / ROIAlign tests, the 1x1 WS-wgrad threshold A/B, then the
# training evidence refresh (PMC, bench line, timed-region profile).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py tests/test_gpu_geometry.py -k "conv or roi or wgrad" > gpurun_out/fa_tests.log 2>&1 \
  || { tail -40 gpurun_out/fa_tests.log; exit 1; }
tail -1 gpurun_out/fa_tests.log
timeout -k 10 300 python -u tools/ws_ab.py --key wgrad_ws1 --arms 6,4,3 --set wgrad --iters 20 --rounds 3 \
  > gpurun_out/ws1_ab.log 2>&1 || { tail -20 gpurun_out/ws1_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ws1_ab.log | tail -10
timeout -k 10 300 python -u tools/ab_inproc.py --switch tune:wgrad_ws1=4,6 --blocks 6 --steps 10 \
  > gpurun_out/ws1_inproc.log 2>&1 || { tail -20 gpurun_out/ws1_inproc.log; exit 1; }
tail -1 gpurun_out/ws1_inproc.log
bash tools/refresh_a.sh r3
