# r6: the whole GPU suite, smoke, and the default bench line on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r6n_gpu_suite.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6n_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r6n_bench.log 2>&1
