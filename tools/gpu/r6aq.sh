# r6: the fused preprocess (d2mi_preprocess_images): its parity test, then a
# same-box A/B of the training step and the RetinaNet inference step, torch's
# five launches (D2MI_FUSED_PREPROCESS=0) vs the one launch, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "preprocess or stem" > gpurun_out/r6aq_tests.log 2>&1 &&
for i in 1 2 3; do
D2MI_FUSED_PREPROCESS=0 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 40 > gpurun_out/r6aq_train_off_$i.log 2>&1 &&
D2MI_FUSED_PREPROCESS=1 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 40 > gpurun_out/r6aq_train_on_$i.log 2>&1 || exit 1
done &&
D2MI_FUSED_PREPROCESS=0 timeout -k 10 300 python -u bench.py --model retinanet_R_101_FPN --mode infer --cpu-baseline 0 > gpurun_out/r6aq_retina_off.log 2>&1 &&
D2MI_FUSED_PREPROCESS=1 timeout -k 10 300 python -u bench.py --model retinanet_R_101_FPN --mode infer --cpu-baseline 0 > gpurun_out/r6aq_retina_on.log 2>&1
