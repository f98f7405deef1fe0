# r6: B[R] split into the mask-branch forward (B1) and the rest: graphed and
# DP tests, then the bench with / without the split, alternating
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_graphed.py tests/test_gpu_dp.py > gpurun_out/r6p_tests.log 2>&1 &&
for i in 1 2 3; do
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 30 --split-b 1 > gpurun_out/r6p_split_$i.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 30 --split-b 0 > gpurun_out/r6p_one_$i.log 2>&1 || exit 1
done
