#!/bin/bash
# r5: stream 1x1 per-shape A/B with the force arm (every eligible shape, TN by
# task count), then the GPU suite and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stream_ab.py --min-m -1 > gpurun_out/r5n_stream_ab.log 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5n_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5n_bench.log 2>&1
