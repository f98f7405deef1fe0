#!/bin/bash
# GPU box: the RPN head's multi-level training form (rpn_levels): its tests,
# the whole -m gpu suite, the in-step A/B, launches per step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu \
  tests/test_gpu_train.py -k "levels or accumulator or whole_training or deterministic" > gpurun_out/levels_tests.log 2>&1 || { grep -E "Error|error|assert|FAILED" gpurun_out/levels_tests.log | head -30; tail -30 gpurun_out/levels_tests.log; exit 1; }
tail -1 gpurun_out/levels_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_levels.log 2>&1
rc=$?
tail -1 gpurun_out/gpu_tests_levels.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests_levels.log | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_inproc.py --switch rpn_levels --blocks 8 --steps 10 \
  > gpurun_out/levels_inproc.log 2>&1 || { tail -20 gpurun_out/levels_inproc.log; exit 1; }
tail -1 gpurun_out/levels_inproc.log
bash tools/profile_bench.sh levels --steps 5 --warmup 3 || exit 1
cat gpurun_out/levels_timed_kernel_stats_summary.json | tr -d '\n'; echo
