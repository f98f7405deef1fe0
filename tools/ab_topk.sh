set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_retinanet.py -x -v --timeout 200 --timeout-method thread -k "retina or topk" > gpurun_out/topk_tests.log 2>&1 || { tail -40 gpurun_out/topk_tests.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/topk_tests.log | tail -12
for v in 0 1; do D2MI_TOPK_FLOOR=$v timeout -k 10 200 python bench.py --model retinanet_R_101_FPN --mode infer --cpu-baseline 0 > gpurun_out/topk_bench_$v.log 2>&1 || exit 1; python -c "import json;d=json.loads(open('gpurun_out/topk_bench_$v.log').read().strip().splitlines()[-1]);print($v,d['value'],d['kernels']['retinanet_postprocess'])"; done
bash tools/profile_bench.sh r2x_retina --model retinanet_R_101_FPN --mode infer --steps 5 --warmup 3 > /dev/null && grep -E "topk" gpurun_out/prof_r2x_retina/run_kernel_stats.csv | cut -c1-70,200-300
