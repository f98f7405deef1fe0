#!/bin/bash
# GPU box: the -m gpu suite, smoke, per-shape + in-step A/B of the wgrad XCD
# order, the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s4.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_s4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s4.log 2>&1 || { tail -20 gpurun_out/smoke_s4.log; exit 1; }
tail -1 gpurun_out/smoke_s4.log
timeout -k 10 300 python -u tools/ws_ab.py --key wgrad_xcd --arms 0,1 --set wgrad --iters 20 --rounds 3 \
  > gpurun_out/wgrad_xcd_ab.log 2>&1 || { tail -20 gpurun_out/wgrad_xcd_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/wgrad_xcd_ab.log | tail -12
timeout -k 10 300 python -u tools/ab_inproc.py --switch tune:wgrad_xcd --blocks 6 --steps 10 \
  > gpurun_out/wgrad_xcd_inproc.log 2>&1 || { tail -20 gpurun_out/wgrad_xcd_inproc.log; exit 1; }
tail -1 gpurun_out/wgrad_xcd_inproc.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_s4.log 2>&1 || { tail -20 gpurun_out/bench_s4.log; exit 1; }
tail -1 gpurun_out/bench_s4.log | cut -c1-700
timeout -k 10 900 bash tools/pmc_traffic.sh s4 > gpurun_out/pmc_s4.log 2>&1 || { tail -5 gpurun_out/pmc_s4.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s4_pmc.json')); print({k: v for k, v in d.items() if 'wgrad' in k or 'conv2d_split' in k})" | cut -c1-900
exit $rc
