#!/bin/bash
# GPU box: the -m gpu parity suite (log in gpurun_out/<tag>_tests.log), then
# the given command -- only if the suite ended normally (all passed, rc 0, or
# an assertion failure, rc 1); a crash, abort, fault or time-out ends here.
# usage: tools/gpu_suite_then.sh <tag> <command...>
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${tag}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
"$@"
