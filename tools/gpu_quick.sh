# GPU suite + the RetinaNet profile's post-processing kernels (run on the box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/profile_bench.sh r2x_retina --model retinanet_R_101_FPN --mode infer --steps 5 --warmup 3 > /dev/null
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_r2x_retina/run_kernel_stats.csv')):
    n = r['Name']
    if any(t in n for t in ('topk', 'retina', 'sort', 'nms')):
        print(f"{r['Calls']:>4} {float(r['AverageNs'])/1000:8.1f} us  {n[:80]}")
PY
tail -1 gpurun_out/prof_r2x_retina.log | cut -c1-200
