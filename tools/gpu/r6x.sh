# r6: RetinaNet post, sixth pass: 720 (208 + the k-th select in DPP) and 1744
# (+ the NMS IoU only where normalised boxes intersect); parity and model
# tests with the tuning forced to 1744 through the environment, the A/B, bench
export TMPDIR=/tmp
mkdir -p gpurun_out
D2MI_RETINA_VAR=1744 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_retinanet.py -k "retinanet_inference or retinanet" > gpurun_out/r6x_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,720,1744 --debug --rounds 7 > gpurun_out/r6x_ab.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/r6x_bench_retinanet.log 2>&1
