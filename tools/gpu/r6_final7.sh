# r6 round end, the final tree (after the FrozenBN backward change): the
# whole GPU suite and smoke
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r6_final7_gpu_suite.log 2>&1 &&
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_final7_smoke.log 2>&1
