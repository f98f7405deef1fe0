export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/graph_audit.py --no-arena > gpurun_out/r5a_audit_noarena.log 2>&1 &&
timeout -k 10 300 python -u tools/graph_audit.py --expect-clean > gpurun_out/r5a_audit_arena.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_graphed.py > gpurun_out/r5a_graphed.log 2>&1
