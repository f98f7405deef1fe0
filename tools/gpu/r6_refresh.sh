# r6 round end, part 2: the evidence refresh (PMC passes, the four bench lines,
# timed-region profiles, conv shapes); large intermediates removed after
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/refresh_profiles.sh r6 > gpurun_out/r6_refresh.log 2>&1
rc=$?
find gpurun_out -name "*.csv" -size +5M -delete
find gpurun_out -name "*.db" -delete
exit $rc
