#!/bin/bash
# GPU box: the RPN 3x3's level weight-gradient accumulator (rpn_conv_acc):
# the bit-identity test, wgrad tests, the whole -m gpu suite, the in-step A/B
# and the launches per step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu \
  tests/test_gpu_train.py -k "accumulator" > gpurun_out/acc_tests.log 2>&1 || { tail -30 gpurun_out/acc_tests.log; exit 1; }
tail -1 gpurun_out/acc_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_acc.log 2>&1
rc=$?
tail -1 gpurun_out/gpu_tests_acc.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests_acc.log | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_inproc.py --switch rpn_conv_acc --blocks 8 --steps 10 \
  > gpurun_out/acc_inproc.log 2>&1 || { tail -20 gpurun_out/acc_inproc.log; exit 1; }
tail -1 gpurun_out/acc_inproc.log
bash tools/profile_bench.sh acc --steps 5 --warmup 3 || exit 1
cat gpurun_out/acc_timed_kernel_stats_summary.json | tr -d '\n'; echo
