#!/bin/bash
# GPU suite + smoke + the default bench line (run on the GPU box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests3.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1 || { tail -20 gpurun_out/smoke3.log; exit 1; }
tail -1 gpurun_out/smoke3.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench3.log 2>&1 || { tail -20 gpurun_out/bench3.log; exit 1; }
tail -1 gpurun_out/bench3.log | cut -c1-600
exit $rc
