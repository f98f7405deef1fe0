# r6: the division-free IoU-above-threshold test (tuning "iou_fast"): the NMS
# / RetinaNet / Fast R-CNN parity tests, then same-box A/Bs (D2MI_IOU_FAST=0
# vs 1) of the RetinaNet inference step and the training step, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "nms or retinanet or fast_rcnn or proposals" > gpurun_out/r6ay_tests.log 2>&1 &&
for i in 1 2; do
D2MI_IOU_FAST=0 timeout -k 10 300 python -u bench.py --model retinanet_R_101_FPN --mode infer --cpu-baseline 0 > gpurun_out/r6ay_retina_off_$i.log 2>&1 &&
D2MI_IOU_FAST=1 timeout -k 10 300 python -u bench.py --model retinanet_R_101_FPN --mode infer --cpu-baseline 0 > gpurun_out/r6ay_retina_on_$i.log 2>&1 || exit 1
done &&
for i in 1 2; do
D2MI_IOU_FAST=0 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 > gpurun_out/r6ay_train_off_$i.log 2>&1 &&
D2MI_IOU_FAST=1 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 > gpurun_out/r6ay_train_on_$i.log 2>&1 || exit 1
done
