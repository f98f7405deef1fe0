# r6: RetinaNet post-processing, third pass: 128 = the finish bitonic in DPP /
# permlane lane permutations, 208 = 16 + 64 + 128; NMS sub-phase stamps.
# Parity tests first ("fused_var208"), then the A/B against var 0
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "retinanet_inference" > gpurun_out/r6t_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,80,128,208 --debug --rounds 7 > gpurun_out/r6t_ab.log 2>&1
