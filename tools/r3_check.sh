set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1 || { tail -20 gpurun_out/smoke2.log; exit 1; }
tail -2 gpurun_out/smoke2.log
timeout -k 10 400 python -u bench.py --mode infer --model faster_rcnn_R_50_FPN > gpurun_out/bench_c2.log 2>&1 || { tail -20 gpurun_out/bench_c2.log; exit 1; }
tail -1 gpurun_out/bench_c2.log | cut -c1-400
timeout -k 10 400 python -u bench.py --mask-fixed-rows --cpu-baseline 0 > gpurun_out/bench_fixedrows.log 2>&1 || { tail -20 gpurun_out/bench_fixedrows.log; exit 1; }
tail -1 gpurun_out/bench_fixedrows.log | cut -c1-400
exit $rc
