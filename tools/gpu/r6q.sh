# r6: RetinaNet post-processing variants (tuning retina_var): 1 = 32 KB collect
# chunks, 2 = rolled bitonic, 4 = warm relaunches (stamps only), 8 = floor
# run cap, 16 = many-workgroup compaction before the finish, 32 = rank +
# NMS folded into the finish.  Parity tests
# first (the variants together as "fused_var59"), then outputs compared to
# var 0 with per-segment phase stamps and times, then the model tests
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "retinanet_inference" > gpurun_out/r6q_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,1,2,4,8,16,32,24,56,57,58 --debug --rounds 5 > gpurun_out/r6q_ab.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_retinanet.py >> gpurun_out/r6q_tests.log 2>&1
