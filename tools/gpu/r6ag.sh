# r6: the RPN merge rank with its score-word fill batched 8 entries a round:
# proposal tests, then a kernel trace of the training bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "rpn or proposal or topk" > gpurun_out/r6ag_tests.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_r6ag -o t -- python bench.py --cpu-baseline 0 --no-kernel-timing --fixed-rows-steps 0 --steps 10 > gpurun_out/r6ag_prof.log 2>&1 &&
python tools/rocpd_stats.py /tmp/prof_r6ag/t_results.db --match "merge_rank|nms_scan|topk" --csv gpurun_out/r6ag_stats.csv
