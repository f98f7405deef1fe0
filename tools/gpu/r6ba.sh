# r6: the batched FrozenBN backward without the gamma sums (gamma constant):
# the fold tests, the training / graphed tests, then a same-box A/B of the
# training step against the library before the change (ab_r6b/libA.so)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train.py -k "fold or frozen or overfits or gradients_reach" > gpurun_out/r6ba_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_graphed.py > gpurun_out/r6ba_graphed_tests.log 2>&1 &&
for i in 1 2 3; do
D2MI_LIB=ab_r6b/libA.so timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 > gpurun_out/r6ba_train_A_$i.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 > gpurun_out/r6ba_train_B_$i.log 2>&1 || exit 1
done
