#!/bin/bash
# ROIAlign backward A/B inside the training step: kernel trace of three short
# bench runs (sort digit width x side-stream clear), the per-kernel timeline of
# the step's backward sequences (tools/roi_bwd_timeline.py), then the bench
# line of each configuration.
export TMPDIR=/tmp; mkdir -p gpurun_out
for cfg in "10 0" "8 0" "8 1"; do
  set -- $cfg
  tag=b$1_ns$2
  if [ "$2" = 1 ]; then export D2MI_NO_SIDE_STREAM=1; else unset D2MI_NO_SIDE_STREAM; fi
  D2MI_SORT_BITS=$1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_$tag.log 2>&1 || exit 2
  f=$(find gpurun_out/prof_$tag -name "*kernel_trace.csv" | head -1)
  python3 tools/roi_bwd_timeline.py $f > gpurun_out/roi_tl_$tag.txt
  find gpurun_out/prof_$tag -name "*trace.csv" -delete
  D2MI_SORT_BITS=$1 timeout -k 10 300 python3 bench.py > gpurun_out/bench_$tag.log 2>&1 || exit 3
done
