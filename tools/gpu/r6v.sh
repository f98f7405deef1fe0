# r6: RetinaNet post with the r6 finish as the default (retina_var 208):
# parity tests (both forms), the model tests, the A/B against the r5 form,
# then the RetinaNet R101 inference bench line
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "retinanet_inference" tests/test_retinanet.py > gpurun_out/r6v_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,208 --debug --rounds 7 > gpurun_out/r6v_ab.log 2>&1 &&
timeout -k 10 400 python -u bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/r6v_bench_retinanet.log 2>&1
