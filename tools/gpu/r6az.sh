# r6: the NMS near-threshold fixture on the final library (both scans)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "iou_at_the_threshold or nms_golden" > gpurun_out/r6az_tests.log 2>&1
