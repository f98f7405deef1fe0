#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_solo.py -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/r4bb_tests.log 2>&1 || { tail -30 gpurun_out/r4bb_tests.log; exit 1; }
tail -1 gpurun_out/r4bb_tests.log
timeout -k 10 400 python3 tools/ab_inproc.py --switch gn_nhwc --model solo_v2_R_50_FPN --blocks 6 --steps 5 > gpurun_out/r4bb_ab.log 2>&1 || { tail -20 gpurun_out/r4bb_ab.log; exit 1; }
tail -1 gpurun_out/r4bb_ab.log
