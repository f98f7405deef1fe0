#!/bin/bash
# Round-4 GPU pass (run on the GPU box): the graphed-step parity test, the
# -m gpu suite, the training bench line eager and graphed, in-process A/Bs of
# the round's switches, the ROIAlign forward's gather ceiling, and a
# same-lease A/B of the r2 / r3 / HEAD trees (ab_r2, ab_r3 by git archive,
# libraries built in the container).  Every GPU step has its own time limit;
# a crash / abort / time-out ends the chain (a test assertion, rc 1, does not).
set -o pipefail
mkdir -p gpurun_out
step() { local ok=$1 t=$2 name=$3; shift 3; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/r4a_$name.log 2>&1; local rc=$?; tail -3 gpurun_out/r4a_$name.log; if [ $rc -ne 0 ] && [ $rc -ne $ok ]; then echo "$name rc=$rc: stopping"; exit $rc; fi; }
step 1 400 graphed python -u -m pytest tests/test_gpu_graphed.py -x -v -s --timeout 300 --timeout-method thread
step 1 600 tests python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --ignore tests/test_gpu_graphed.py
step 0 300 bench_eager python3 -u bench.py --graphs 0 --cpu-baseline 0
step 0 300 bench python3 -u bench.py --graphs 1 --cpu-baseline 0
step 0 300 ab_coop python3 -u tools/ab_inproc.py --switch tune:conv_coop=1,0 --blocks 6
step 0 300 ab_defer python3 -u tools/ab_inproc.py --switch defer_pixels --blocks 6
step 0 200 gather python3 -u tools/gather_ceiling.py
bash tools/ab_tree.sh 2 r4a_trees ab_r2 ab_r3 . 2>&1 | tail -8
