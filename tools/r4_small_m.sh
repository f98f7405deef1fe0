#!/bin/bash
# Per-shape A/B of the split policy knobs on the small-M (res4 / res5 / p4-p6)
# conv shapes, one process per setting (the knobs are read once per process).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r4n_small_m.log
: > $out
for cfg in "base:" "mink40:D2MI_CONV_WS_MINK=40" "slots256:D2MI_CONV_SPLIT_SLOTS=256" \
           "slots1024:D2MI_CONV_SPLIT_SLOTS=1024" "slots2048:D2MI_CONV_SPLIT_SLOTS=2048" \
           "wslots512:D2MI_WGRAD_SLOTS=512" "wslots1024:D2MI_WGRAD_SLOTS=1024" "wminch8:D2MI_WGRAD_MINCH=8" "base2:"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  echo "== $name $envs" >> $out
  env $envs timeout -k 10 120 python3 tools/conv_ab.py --set small_m --iters 40 >> $out 2>&1 || exit 1
done
cat $out | grep -v amdgpu.ids
