# r6: kernel trace of the RetinaNet post A/B tool (default variant): per-kernel
# durations, to split the rank phase into kernel time and launch boundaries
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_rp -o rp -- python tools/retina_post_ab.py --vars 3792 --rounds 3 > gpurun_out/r6_rp_run.log 2>&1 &&
python tools/rocpd_stats.py /tmp/prof_rp/rp_results.db --csv gpurun_out/r6_rp_stats.csv > gpurun_out/r6_rp_stats.log 2>&1
