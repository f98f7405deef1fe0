# r6: the ROI-head sampling glue on d2mi_roi_gt_classes / d2mi_roi_sample_take:
# its parity test, the graphed-vs-eager and data-parallel training tests, then
# a same-box A/B of the training step (D2MI_FUSED_SAMPLE_TAKE=0 vs 1), alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "sample_take or preprocess" > gpurun_out/r6as_tests.log 2>&1 &&
timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_graphed.py tests/test_gpu_train.py tests/test_gpu_dp.py > gpurun_out/r6as_train_tests.log 2>&1 &&
for i in 1 2 3; do
D2MI_FUSED_SAMPLE_TAKE=0 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 40 > gpurun_out/r6as_train_off_$i.log 2>&1 &&
D2MI_FUSED_SAMPLE_TAKE=1 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 40 > gpurun_out/r6as_train_on_$i.log 2>&1 || exit 1
done
