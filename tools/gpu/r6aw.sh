# r6: what the bench line's event-timed sample step (one eager step with HIP
# events around every hot launch, inside the timed region: the live roofline)
# costs the throughput: default vs --no-kernel-timing, alternating on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 > gpurun_out/r6aw_default_$i.log 2>&1 &&
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --no-kernel-timing > gpurun_out/r6aw_notiming_$i.log 2>&1 || exit 1
done
