# r6: int8-MFMA Matrix NMS v3 + the compensation max folded into the reduce:
# SOLO tail tests (both paths), then a kernel trace of the C5 bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_solo.py -k "tail" > gpurun_out/r6h_solo.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6h_solo -o r6h -- python bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 --steps 5 > gpurun_out/r6h_solo_prof.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 > gpurun_out/r6h_solo_bench_mfma.log 2>&1
