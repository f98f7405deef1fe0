# r6: RetinaNet post, eighth pass: 7888 = 3792 + no rank launch (the NMS ranks
# each 128-candidate window itself); parity and model tests with 7888 forced,
# the A/B, the bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
D2MI_RETINA_VAR=7888 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_retinanet.py -k "retinanet_inference or retinanet" > gpurun_out/r6aa_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,3792,7888 --debug --rounds 7 > gpurun_out/r6aa_ab.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/r6aa_bench_retinanet.log 2>&1
