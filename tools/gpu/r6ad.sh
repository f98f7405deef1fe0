# r6: RetinaNet post, the floor's ts-th maximum by a workgroup radix select
# (retina_var 8192): parity + model tests with 16080 forced, the A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
D2MI_RETINA_VAR=16080 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_retinanet.py -k "retinanet_inference or retinanet" > gpurun_out/r6ad_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,7888,16080 --debug --rounds 7 > gpurun_out/r6ad_ab.log 2>&1
