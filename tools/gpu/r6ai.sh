# r6: same-box A/B of the training step, library A (before) vs B (the split-K
# reduce's float4 epilogue + 32-bit indexing, the resample gradients' 32-bit
# indexing), alternating three times; first the resample / conv tests on B
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "upsample or stride_scatter or scatter or conv" > gpurun_out/r6ai_tests.log 2>&1 &&
for i in 1 2 3; do
D2MI_LIB=ab_r6/libA.so timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 40 > gpurun_out/r6ai_A_$i.log 2>&1 &&
D2MI_LIB=ab_r6/libB.so timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 40 > gpurun_out/r6ai_B_$i.log 2>&1 || exit 1
done
