#!/bin/bash
# Round-4 GPU pass: the whole -m gpu suite on the current tree, then
# timed-region kernel profiles of the training bench for HEAD and the r3 tree
# (ab_r3: per-kernel comparison of the two rounds on one box), then the
# training bench line.  A crash / abort / time-out ends the chain.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r4g}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "suite rc=$rc: stopping"; exit $rc; fi
bash tools/profile_bench.sh ${T}_head --steps 5 --warmup 3 || exit $?
(cd ab_r3 && bash tools/profile_bench.sh ${T}_r3 --steps 5 --warmup 3) || exit $?
cp ab_r3/gpurun_out/${T}_r3_timed_kernel_stats.csv gpurun_out/ 2>/dev/null
timeout -k 10 400 python3 bench.py > gpurun_out/${T}_bench_train.log 2>&1 || exit $?
tail -1 gpurun_out/${T}_bench_train.log | cut -c1-400
