#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "rpn or train_step or whole or level" \
    --timeout 300 --timeout-method thread > gpurun_out/r4w_tests.log 2>&1 || { tail -30 gpurun_out/r4w_tests.log; exit 1; }
tail -1 gpurun_out/r4w_tests.log
timeout -k 10 300 python3 tools/ab_inproc.py --switch skinny_levels --blocks 10 --steps 10 > gpurun_out/r4w_ab.log 2>&1 || exit 1
tail -1 gpurun_out/r4w_ab.log
