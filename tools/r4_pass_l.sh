#!/bin/bash
# ROIAlign pixel-pass change: its exactness tests, then the timed-region
# profile of the training bench (roi_bwd_pixel time per step).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "roi or deferred or train_step or whole" \
    --timeout 300 --timeout-method thread > gpurun_out/r4l_tests.log 2>&1 || { tail -30 gpurun_out/r4l_tests.log; exit 1; }
tail -2 gpurun_out/r4l_tests.log
STEPS=10 bash tools/profile_bench.sh r4l_pix
grep -i "roi_bwd_pixel" gpurun_out/r4l_pix_timed_kernel_stats.csv | cut -c1-60,150-260
