#!/bin/bash
# Round-end evidence on the GPU box: the whole -m gpu suite (log kept), the
# smoke, the training refresh (PMC, bench line, timed-region profile), the
# host enqueue time.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_tests.txt 2>&1
rc=$?
tail -1 gpurun_out/r3_gpu_tests.txt
grep -E "FAILED|ERROR" gpurun_out/r3_gpu_tests.txt | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -1 gpurun_out/r3_smoke.log
bash tools/refresh_a.sh r3 || exit 1
timeout -k 10 300 python -u tools/host_time.py --mode train --steps 7 > gpurun_out/r3_host_time.log 2>&1 || { tail -20 gpurun_out/r3_host_time.log; exit 1; }
tail -1 gpurun_out/r3_host_time.log
