#!/bin/bash
set -o pipefail
tag=${1:-stem}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "stem or train_step or whole" \
    --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
STEPS=10 bash tools/profile_bench.sh ${tag}
grep -i "stem_" gpurun_out/${tag}_timed_kernel_stats.csv | cut -d, -f1-4 | cut -c1-120
