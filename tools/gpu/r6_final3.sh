# r6 round end, the final tree (after the late RetinaNet floor / rank /
# merge-rank changes): the whole GPU suite, smoke, and the default bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r6_final3_gpu_suite.log 2>&1 &&
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_final3_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r6_final3_bench.log 2>&1
