#!/bin/bash
# The bench's data-parallel path (torchrun, 2 ranks, bucketed all-reduce,
# barrier + max-over-ranks timing; r6: graph-replayed, the all-reduces
# between the backward and update graphs) rehearsed on a 1-GPU box: both
# ranks on cuda:0 over gloo (D2MI_REHEARSE_ONE_GPU=1) -- a code-path check,
# never a measurement.   usage: tools/dp_rehearse.sh [log name]
set -o pipefail
mkdir -p gpurun_out
log=gpurun_out/${1:-dp_rehearse}.log
D2MI_REHEARSE_ONE_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 \
    --warmup 2 --cpu-baseline 0 --fixed-rows-steps 0 > $log 2>&1 || { tail -30 $log; exit 1; }
tail -1 $log | cut -c1-600
