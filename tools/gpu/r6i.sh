# r6: ROIAlign forward variants (one wave iteration per wave, U = 4 / 2 / 8)
# on the step's own box-pooler inputs, cold caches, beside the gather ceilings
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/gather_ceiling.py --iters 20 --rounds 5 > gpurun_out/r6i_gather_ceiling.log 2>&1
