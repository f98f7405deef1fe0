#!/bin/bash
# Round-end rehearsal: the whole -m gpu suite, smoke(), the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/r4y_tests.log 2>&1 || { tail -30 gpurun_out/r4y_tests.log; exit 1; }
tail -1 gpurun_out/r4y_tests.log
bash tools/final_check.sh
