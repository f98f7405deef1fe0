# r6: RetinaNet post, fifth pass: 208 (default) + 256 (collect loads not gated
# on the info words) / + 512 (k-th select in DPP / permlane) / both; the
# parity and model tests, the A/B, the R101 inference bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_retinanet.py -k "retinanet_inference or retinanet" > gpurun_out/r6w_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,208,464,720,976 --debug --rounds 7 > gpurun_out/r6w_ab.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/r6w_bench_retinanet.log 2>&1
