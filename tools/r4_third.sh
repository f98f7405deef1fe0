#!/bin/bash
# Round-4 GPU pass 3 (no graph replay anywhere): the captured graphs dumped
# as DOT files (tools/graph_dump.py) to find what faulted the first replay,
# the ROIAlign-backward / RetinaNet / NMS tests, the eager bench line, the
# conv_coop / defer_pixels in-process A/Bs, the ROIAlign gather ceiling and
# the r2 / r3 / HEAD tree A/B.  A crash / abort / time-out ends the chain.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r4d}
step() { local ok=$1 t=$2 name=$3; shift 3; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; tail -3 gpurun_out/${T}_$name.log; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then echo "$name rc=$rc: stopping"; exit $rc; fi; }

step 1 500 roi python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train.py -k "roi or deferred or whole_training"
step 0 300 bench python3 -u bench.py --cpu-baseline 0
step 0 300 ab_coop python3 -u tools/ab_inproc.py --switch tune:conv_coop=1,0 --blocks 6
step 0 300 ab_defer python3 -u tools/ab_inproc.py --switch defer_pixels --blocks 6
step 0 200 gather python3 -u tools/gather_ceiling.py
bash tools/ab_tree.sh 2 ${T}_trees ab_r2 ab_r3 . 2>&1 | tail -8
