# r6: Matrix NMS on 128 x 128 workgroup tiles with the bits expanded once into
# LDS (tuning solo_mfma 3): SOLO tail tests (all paths), then a kernel trace
# of the C5 bench for modes 2 and 3 (stats only: the databases stay on the box)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_solo.py -k "tail" > gpurun_out/r6ae_solo.log 2>&1 &&
for m in 2 3; do
D2MI_SOLO_MFMA=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_r6ae_$m -o m$m -- python bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 --steps 5 > gpurun_out/r6ae_prof_$m.log 2>&1 &&
python tools/rocpd_stats.py /tmp/prof_r6ae_$m/m${m}_results.db --match "solo" --csv gpurun_out/r6ae_stats_$m.csv || exit 1
done
