#!/bin/bash
# r5: ROIAlign backward in 5 + 4 launches (one emit for both sets, long sort +
# segments fused): parity, then the bench line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "roi or deferred or grad_share or whole_training or dp" > gpurun_out/r5zf_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py --cpu-baseline 0 > gpurun_out/r5zf_bench.log 2>&1
