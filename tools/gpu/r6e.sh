# r6: the int8-MFMA Matrix NMS v2 (LDS-staged rows, transposed IoU rows):
# SOLO tail tests (both paths), the C5 bench line each way, a kernel trace of
# the MFMA arm; then the gather-ceiling tool with the guide-shaped gather
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_solo.py -k "tail" > gpurun_out/r6e_solo.log 2>&1 &&
D2MI_SOLO_MFMA=1 timeout -k 10 300 python -u bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 > gpurun_out/r6e_solo_bench_mfma.log 2>&1 &&
D2MI_SOLO_MFMA=0 timeout -k 10 300 python -u bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 > gpurun_out/r6e_solo_bench_popcount.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6e_solo -o r6e -- python bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 --steps 5 > gpurun_out/r6e_solo_prof.log 2>&1 &&
timeout -k 10 400 python -u tools/gather_ceiling.py --iters 20 --rounds 3 > gpurun_out/r6e_gather_ceiling.log 2>&1
