#!/bin/bash
# Kernel-trace profile of bench.py's timed region (run on the GPU box).
# usage: tools/profile_bench.sh <tag> [bench args...]
set -eo pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
export TMPDIR=/tmp
rm -rf "$out"
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d "$out" -o run \
    -- python3 bench.py --cpu-baseline 0 --no-kernel-timing "$@" > "$out.log" 2>&1
python3 tools/prof_window.py "$out" "gpurun_out/${tag}_timed_kernel_stats.csv" --steps "${STEPS:-5}"
find "$out" -name "*trace.csv" -delete
find "$out" -name "*.db" -delete
tail -1 "$out.log"
