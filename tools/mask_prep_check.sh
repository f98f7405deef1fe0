#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "train or mask or whole" \
    --timeout 300 --timeout-method thread > gpurun_out/r4v_tests.log 2>&1 || { tail -30 gpurun_out/r4v_tests.log; exit 1; }
tail -1 gpurun_out/r4v_tests.log
timeout -k 10 300 python3 tools/ab_inproc.py --switch mask_prep_early --blocks 10 --steps 10 > gpurun_out/r4v_ab.log 2>&1 || exit 1
tail -1 gpurun_out/r4v_ab.log
