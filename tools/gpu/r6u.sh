# r6: RetinaNet post-processing, fourth pass: 208 (r6t's best) plus the collect
# grid as long as the chunks (256) or half the resident workgroups (512), and
# the box-delta prefetch under the sort (1024).  Parity tests first
# ("fused_var1488"), then the A/B against var 0
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "retinanet_inference" > gpurun_out/r6u_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,208,464,720,1232,1488 --debug --rounds 7 > gpurun_out/r6u_ab.log 2>&1
