#!/bin/bash
# r5: ROIAlign backward (touched entries carry runs, scratch-free touched
# range, 2-row batch variant): parity, in-step A/B of roi_bwd_rec 1 / 2 / 0,
# and the widened stream 1x1 selection against the tiled kernel in-step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "roi or deferred" > gpurun_out/r5w_tests.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_inproc.py --switch tune:roi_bwd_rec=1,2 --blocks 10 --steps 10 > gpurun_out/r5w_ab_rb.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_inproc.py --switch tune:roi_bwd_rec=1,0 --blocks 10 --steps 10 > gpurun_out/r5w_ab_rec.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_inproc.py --switch tune:conv_stream=8192,0 --blocks 10 --steps 10 > gpurun_out/r5w_ab_stream.log 2>&1
