#!/bin/bash
# The -m gpu suite (with the SOLOv2 training test), then the SOLOv2 training
# bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_solo.py -m gpu -q -x -k training \
    --timeout 300 --timeout-method thread > gpurun_out/r4m_solo_train_test.log 2>&1 || { tail -40 gpurun_out/r4m_solo_train_test.log; exit 1; }
tail -2 gpurun_out/r4m_solo_train_test.log
timeout -k 10 400 python3 bench.py --model solo_v2_R_50_FPN --mode train --cpu-baseline 0 > gpurun_out/r4m_bench_solo_train.log 2>&1 || { tail -30 gpurun_out/r4m_bench_solo_train.log; exit 1; }
tail -1 gpurun_out/r4m_bench_solo_train.log | cut -c1-300
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    > gpurun_out/r4m_tests.log 2>&1 || { tail -30 gpurun_out/r4m_tests.log; exit 1; }
tail -2 gpurun_out/r4m_tests.log
