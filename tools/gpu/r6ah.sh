# r6: split-K reduce with the float4 epilogue and 32-bit indexing: conv and
# training tests (results bit-identical), a kernel trace of the training bench
# (reduce kernels' times), then two bench lines
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train.py tests/test_gpu_graphed.py -k "conv or train or graphed or wgrad" > gpurun_out/r6ah_tests.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_r6ah -o t -- python bench.py --cpu-baseline 0 --no-kernel-timing --fixed-rows-steps 0 --steps 10 > gpurun_out/r6ah_prof.log 2>&1 &&
python tools/rocpd_stats.py /tmp/prof_r6ah/t_results.db --match "reduce" --csv gpurun_out/r6ah_stats.csv &&
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 > gpurun_out/r6ah_bench_1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 > gpurun_out/r6ah_bench_2.log 2>&1
