#!/bin/bash
# GPU-box check: the -m gpu parity suite, then the default bench line.
# A test assertion failure (rc 1) still lets the bench run; a crash, abort,
# fault or time-out (any other rc) ends the script there.
mkdir -p gpurun_out
timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -v --timeout 300 \
    --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ -n "$NO_BENCH" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-450} python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_default.log 2>&1
brc=$?
tail -1 gpurun_out/bench_default.log
exit $(( rc > brc ? rc : brc ))
