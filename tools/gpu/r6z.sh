# r6: RetinaNet post, seventh pass: 3792 = 1744 + the NMS tile resolved as a
# ballot fixed point over column words; parity and model tests with 3792
# forced through the environment, the A/B, the bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
D2MI_RETINA_VAR=3792 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_retinanet.py -k "retinanet_inference or retinanet" > gpurun_out/r6z_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,1744,3792 --debug --rounds 7 > gpurun_out/r6z_ab.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/r6z_bench_retinanet.log 2>&1
