#!/bin/bash
# Host-time pass: the -m gpu suite, host time of the training step, the
# training bench line and its timed-region kernel profile (with idle gaps).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/r4k_tests.log 2>&1 || { tail -30 gpurun_out/r4k_tests.log; exit 1; }
tail -2 gpurun_out/r4k_tests.log
timeout -k 10 300 python3 -u tools/host_time.py --steps 9 > gpurun_out/r4k_host_time.log 2>&1 || exit 1
tail -1 gpurun_out/r4k_host_time.log
timeout -k 10 400 python3 bench.py --cpu-baseline 0 > gpurun_out/r4k_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r4k_bench.log | cut -c1-200
STEPS=10 bash tools/profile_bench.sh r4k_head
head -1 gpurun_out/r4k_head_timed_kernel_stats_gaps.txt
