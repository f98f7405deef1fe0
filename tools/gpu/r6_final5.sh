# r6 round end, the final tree (after the FPN top-down hand-off and the
# 60-step bench default): the whole GPU suite, smoke, and the bench lines of
# the four workloads
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r6_final5_gpu_suite.log 2>&1 &&
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_final5_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r6_final5_bench.log 2>&1 &&
timeout -k 10 400 python -u bench.py --mode infer > gpurun_out/r6_final5_bench_infer.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/r6_final5_bench_retinanet.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model solo_v2_R_50_FPN --mode infer > gpurun_out/r6_final5_bench_solo.log 2>&1
