#!/bin/bash
# GPU box: RPN-loss scale folding + mini-mask glue: loss tests, the whole -m
# gpu suite, launches per step, host time.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu \
  tests/test_gpu_train.py tests/test_gpu_ops.py tests/test_gpu_geometry.py -k "rpn_loss or accumulator or whole_training or mask or match or deterministic or dp" > gpurun_out/glue4_tests.log 2>&1 || { tail -30 gpurun_out/glue4_tests.log; exit 1; }
tail -1 gpurun_out/glue4_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_glue4.log 2>&1
rc=$?
tail -1 gpurun_out/gpu_tests_glue4.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests_glue4.log | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/profile_bench.sh glue4 --steps 5 --warmup 3 || exit 1
cat gpurun_out/glue4_timed_kernel_stats_summary.json | tr -d '\n'; echo
timeout -k 10 300 python -u tools/host_time.py --mode train --steps 7 > gpurun_out/host_time_glue4.log 2>&1 || { tail -20 gpurun_out/host_time_glue4.log; exit 1; }
tail -1 gpurun_out/host_time_glue4.log
