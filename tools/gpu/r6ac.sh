# r6: RetinaNet post, the finish's compacted gather locating each entry's
# part by binary search; parity + model tests, the A/B against the r5 form
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_retinanet.py -k "retinanet_inference or retinanet" > gpurun_out/r6ac_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,7888 --debug --rounds 7 > gpurun_out/r6ac_ab.log 2>&1
