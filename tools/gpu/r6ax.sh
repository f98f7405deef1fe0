# r6: the mask head's logit shuffle (predictor before the pixel shuffle):
# its test, the mask / training / graphed tests, then a same-box A/B of the
# training step (D2MI_MASK_SHUFFLE_LOGITS=0 vs 1), alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py -k "shuffle or mask or overfits or gradients_reach" > gpurun_out/r6ax_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_graphed.py > gpurun_out/r6ax_graphed_tests.log 2>&1 &&
for i in 1 2 3; do
D2MI_MASK_SHUFFLE_LOGITS=0 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 40 > gpurun_out/r6ax_train_off_$i.log 2>&1 &&
D2MI_MASK_SHUFFLE_LOGITS=1 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 40 > gpurun_out/r6ax_train_on_$i.log 2>&1 || exit 1
done
