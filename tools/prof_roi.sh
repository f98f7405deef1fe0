export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_roi -o run -- python3 tools/bench_kernels.py --only roi --iters 10 > gpurun_out/prof_roi.log 2>&1
rc=$?
find gpurun_out/prof_roi -name "*trace.csv" -delete
exit $rc
