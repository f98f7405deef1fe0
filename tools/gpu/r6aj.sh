# r6: the RPN matcher's best-GT pass with 16 boxes per thread (4x fewer
# workgroups and per-GT atomics): matcher / sampling / training tests, then a
# kernel trace of the training bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train.py -k "match or sample or train or stride_scatter or upsample" > gpurun_out/r6aj_tests.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_r6aj -o t -- python bench.py --cpu-baseline 0 --no-kernel-timing --fixed-rows-steps 0 --steps 10 > gpurun_out/r6aj_prof.log 2>&1 &&
python tools/rocpd_stats.py /tmp/prof_r6aj/t_results.db --csv gpurun_out/r6aj_stats.csv
