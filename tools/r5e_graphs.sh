# r5: op census of the captures, graphed tests, eager vs graphed training bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/graph_audit.py --ops --expect-clean > gpurun_out/r5e_audit_ops.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_graphed.py > gpurun_out/r5e_graphed.log 2>&1 &&
timeout -k 10 400 python -u bench.py --cpu-baseline 0 > gpurun_out/r5e_bench_eager.log 2>&1 &&
timeout -k 10 400 python -u bench.py --cpu-baseline 0 --graphs 1 --fixed-rows-steps 0 > gpurun_out/r5e_bench_graphs.log 2>&1
