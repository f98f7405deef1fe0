# r6: ROIAlign forward corner loads non-temporal (roi_fwd bit 64) vs default,
# in-step (the bench's per-launch events), alternating arms on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 20 > gpurun_out/r6j_def_$i.log 2>&1 &&
D2MI_ROI_FWD=79 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 20 > gpurun_out/r6j_ntl_$i.log 2>&1 || exit 1
done
