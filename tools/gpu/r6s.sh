# r6: RetinaNet post-processing, second pass (tuning retina_var): 16 = the
# many-workgroup compaction before the finish, 64 = the finish's k-th select
# stopped at the first bound leaving <= 1,024 keys, 80 = both, 4 = warm
# relaunches (stamps only); sub-phase stamps of the sort and the NMS.  Parity
# tests first ("fused_var80"), then the A/B with outputs compared to var 0
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "retinanet_inference" > gpurun_out/r6s_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,4,16,64,80 --debug --rounds 7 > gpurun_out/r6s_ab.log 2>&1
