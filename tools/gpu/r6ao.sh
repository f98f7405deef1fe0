# r6: the RetinaNet R101 inference line and its timed-region kernel profile
# with the final post-processing default (retina_var 12018)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --model retinanet_R_101_FPN --mode infer > gpurun_out/r6ao_bench_retinanet.log 2>&1 &&
bash tools/profile_bench.sh r6ao_retinanet --model retinanet_R_101_FPN --mode infer --steps 5 --warmup 3 > gpurun_out/r6ao_prof.log 2>&1
rc=$?
find gpurun_out -name "*.csv" -size +5M -delete
exit $rc
