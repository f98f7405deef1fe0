#!/bin/bash
# Round-4 GPU pass 2: the new paths' tests (graphed step, RCCL + graphs,
# RetinaNet training, the one-barrier NMS scan), the graphed training bench
# line, the conv_coop / defer_pixels in-process A/Bs, the ROIAlign gather
# ceiling and the r2 / r3 / HEAD tree A/B.  A crash / abort / time-out ends
# the chain (a test assertion, rc 1, does not).
set -o pipefail
mkdir -p gpurun_out
step() { local ok=$1 t=$2 name=$3; shift 3; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/${TAG:-r4b}_$name.log 2>&1; local rc=$?; tail -3 gpurun_out/${TAG:-r4b}_$name.log; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then echo "$name rc=$rc: stopping"; exit $rc; fi; }
step 1 500 newtests python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_graphed.py "tests/test_gpu_dp.py::test_rccl_backend_one_rank_runs_the_reducer" -k "graphed or rccl"
step 1 400 nms python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_geometry.py -k "nms or fast_rcnn or proposals or rpn"
step 1 400 retina python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_retinanet.py -k "training or fused_loss"
step 1 500 roi python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train.py -k "roi or deferred or whole_training"
step 0 300 bench python3 -u bench.py --graphs 1 --cpu-baseline 0
step 0 300 ab_coop python3 -u tools/ab_inproc.py --switch tune:conv_coop=1,0 --blocks 6
step 0 300 ab_defer python3 -u tools/ab_inproc.py --switch defer_pixels --blocks 6
step 0 200 gather python3 -u tools/gather_ceiling.py
bash tools/ab_tree.sh 2 ${TAG:-r4b}_trees ab_r2 ab_r3 . 2>&1 | tail -8
