#!/bin/bash
# In-process step A/Bs of the runtime kernel-selection keys against their
# defaults (errors.hip kTuneDefault), one process per key pair.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r4t_tune_sweep.log
: > $out
for sw in "conv_ws_mink=8,16" "conv_ws_mink=24,16" "wgrad_ws1=4,6" "wgrad_ws1=8,6" "conv_epi=0,1" \
          "wgrad_inc=0,1" "conv_xcd=0,1" "wgrad_xcd=0,1"; do
  timeout -k 10 240 python3 tools/ab_inproc.py --switch tune:$sw --blocks 6 --steps 10 > gpurun_out/r4t_$sw.log 2>&1 || exit 1
  tail -1 gpurun_out/r4t_$sw.log >> $out
done
cat $out
