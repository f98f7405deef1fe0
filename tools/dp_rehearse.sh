#!/bin/bash
# The bench's data-parallel path (torchrun, 2 ranks, bucketed all-reduce,
# barrier + max-over-ranks timing) rehearsed on a 1-GPU box: both ranks on
# cuda:0 over gloo (D2MI_REHEARSE_ONE_GPU=1) -- a code-path check, never a
# measurement.
set -o pipefail
mkdir -p gpurun_out
D2MI_REHEARSE_ONE_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 \
    --warmup 1 --cpu-baseline 0 > gpurun_out/r4q_dp_rehearse.log 2>&1 || { tail -30 gpurun_out/r4q_dp_rehearse.log; exit 1; }
tail -1 gpurun_out/r4q_dp_rehearse.log | cut -c1-400
