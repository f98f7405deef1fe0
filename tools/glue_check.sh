#!/bin/bash
# GPU box: the whole -m gpu suite, then the timed-region kernel profile of the
# training bench (launches per step) and the host enqueue time.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_glue.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_glue.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests_glue.log | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/profile_bench.sh glue --steps 5 --warmup 3 || exit 1
cat gpurun_out/glue_timed_kernel_stats_summary.json 2>/dev/null | cut -c1-600
timeout -k 10 300 python -u tools/host_time.py --mode train --steps 5 > gpurun_out/host_time_glue.log 2>&1 || { tail -20 gpurun_out/host_time_glue.log; exit 1; }
tail -4 gpurun_out/host_time_glue.log
