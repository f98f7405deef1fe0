export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread -k "roi or train or step or sort" > gpurun_out/t_roi.log 2>&1 || { tail -30 gpurun_out/t_roi.log; exit 1; }
tail -1 gpurun_out/t_roi.log
for b in 10 8; do
  D2MI_SORT_BITS=$b timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_roi$b -o run -- python3 tools/bench_kernels.py --only roi --iters 10 > gpurun_out/prof_roi$b.log 2>&1 || exit 2
  f=$(find gpurun_out/prof_roi$b -name "*kernel_trace.csv" | head -1)
  python3 tools/roi_bwd_timeline.py $f > gpurun_out/roi_tl$b.txt
  find gpurun_out/prof_roi$b -name "*trace.csv" -delete
  grep bwd gpurun_out/prof_roi$b.log
done
for b in 10 8; do D2MI_SORT_BITS=$b timeout -k 10 300 python -u bench.py > gpurun_out/b_bits$b.log 2>&1 || exit 3; done
