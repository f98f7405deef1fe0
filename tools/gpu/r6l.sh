# r6: weight gradients on a side stream inside the captured backward: the
# graphed tests (bit-identical to eager), then the bench with / without it
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_graphed.py > gpurun_out/r6l_graphed.log 2>&1 &&
for i in 1 2; do
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 20 --wgrad-side 1 > gpurun_out/r6l_side_$i.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 20 --wgrad-side 0 > gpurun_out/r6l_one_$i.log 2>&1 || exit 1
done
