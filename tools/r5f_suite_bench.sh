# r5: the whole GPU suite, then the default bench line (graphs at N=1, CPU baseline, fixed rows)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r5f_bench.log 2>&1
