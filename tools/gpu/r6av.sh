# r6: kernel-trace profile of the final tree's training bench (timed-region
# per-kernel stats, the rocprof counterpart of the bench line's roofline)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r6av_bench.log 2>&1 &&
bash tools/profile_bench.sh r6av_train --steps 5 --warmup 3 > gpurun_out/r6av_prof.log 2>&1
rc=$?
find gpurun_out -name "*.csv" -size +5M -delete
exit $rc
