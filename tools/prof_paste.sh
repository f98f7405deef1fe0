#!/bin/bash
# Kernel trace of the paste micro-benchmark (kernel time without host overhead).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_paste -o run -- python3 tools/bench_kernels.py --only paste,roi --iters 10 > gpurun_out/prof_paste.log 2>&1
rc=$?
find gpurun_out/prof_paste -name "*trace.csv" -delete
exit $rc
