#!/bin/bash
# Python's cyclic GC and the training step: in-process step A/B (gc disabled
# vs enabled) and host time both ways.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python3 tools/ab_inproc.py --switch gc_off --blocks 8 --steps 10 > gpurun_out/r4u_gc_ab.log 2>&1 || exit 1
tail -1 gpurun_out/r4u_gc_ab.log
timeout -k 10 240 python3 tools/host_time.py --steps 15 > gpurun_out/r4u_host_gc_on.log 2>&1 || exit 1
tail -1 gpurun_out/r4u_host_gc_on.log
timeout -k 10 240 python3 tools/host_time.py --steps 15 --gc-off > gpurun_out/r4u_host_gc_off.log 2>&1 || exit 1
tail -1 gpurun_out/r4u_host_gc_off.log
