#!/bin/bash
# Round-4 GPU pass: the whole -m gpu suite, the ROIAlign pixel-pass grid-cap
# A/B, and the timed-region kernel profile of the training bench.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r4h}
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 -u tools/ab_inproc.py --switch tune:roi_pix_grid=2048,8192 --blocks 6 > gpurun_out/${T}_ab_pix2048.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_ab_pix2048.log
timeout -k 10 300 python3 -u tools/ab_inproc.py --switch tune:roi_pix_grid=512,8192 --blocks 6 > gpurun_out/${T}_ab_pix512.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_ab_pix512.log
bash tools/profile_bench.sh ${T}_head --steps 5 --warmup 3 || exit $?
