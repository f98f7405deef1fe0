# r6 round end: the whole GPU suite, smoke, then the evidence refresh (PMC
# passes, the four bench lines, timed-region profiles, conv shapes); large
# intermediate files are removed so the merge-back stays small
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r6_final_gpu_suite.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_final_smoke.log 2>&1 &&
bash tools/refresh_profiles.sh r6 > gpurun_out/r6_final_refresh.log 2>&1
rc=$?
find gpurun_out -name "*.csv" -size +5M -delete
find gpurun_out -name "*.db" -delete
exit $rc
