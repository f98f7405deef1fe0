# r6: kernel-trace stats of the batched FrozenBN backward, before (ab_r6b/libA.so)
# and after the gamma-sum skip
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && cd - > /dev/null
D2MI_LIB=ab_r6b/libA.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6bb_A -o run -- python3 bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 10 --no-kernel-timing > gpurun_out/r6bb_A.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6bb_B -o run -- python3 bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 10 --no-kernel-timing > gpurun_out/r6bb_B.log 2>&1
rc=$?
find gpurun_out/r6bb_A gpurun_out/r6bb_B -name "*kernel_trace.csv" -delete
exit $rc
