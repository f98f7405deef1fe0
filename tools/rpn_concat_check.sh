#!/bin/bash
# GPU box: the whole -m gpu suite, then the in-step A/B of the RPN head's
# concatenated output layout (rpn_concat).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_rc.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_rc.log
grep -E "FAILED|ERROR" gpurun_out/gpu_tests_rc.log | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_inproc.py --switch rpn_concat --blocks 6 --steps 10 \
  > gpurun_out/rpn_concat_inproc.log 2>&1 || { tail -20 gpurun_out/rpn_concat_inproc.log; exit 1; }
tail -1 gpurun_out/rpn_concat_inproc.log
