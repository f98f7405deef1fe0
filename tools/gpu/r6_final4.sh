# r6 round end, the final tree (after the fused preprocess and the ROI
# sampling glue): the whole GPU suite, smoke, the default bench line, and the
# RetinaNet inference line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r6_final4_gpu_suite.log 2>&1 &&
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_final4_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r6_final4_bench.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/r6_final4_bench_retinanet.log 2>&1
