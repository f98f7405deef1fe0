#!/bin/bash
# GPU box: the WS weight-gradient stagers' pixel cursor (tuning wgrad_inc):
# wgrad tests, per-shape A/B with bit-identity, in-step A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py tests/test_gpu_train.py -k "wgrad or training_step" > gpurun_out/winc_tests.log 2>&1 \
  || { tail -40 gpurun_out/winc_tests.log; exit 1; }
tail -1 gpurun_out/winc_tests.log
timeout -k 10 300 python -u tools/ws_ab.py --key wgrad_inc --arms 0,1 --set wgrad --iters 20 --rounds 3 \
  > gpurun_out/winc_ab.log 2>&1 || { tail -20 gpurun_out/winc_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/winc_ab.log | tail -11
timeout -k 10 300 python -u tools/ab_inproc.py --switch tune:wgrad_inc --blocks 6 --steps 10 \
  > gpurun_out/winc_inproc.log 2>&1 || { tail -20 gpurun_out/winc_inproc.log; exit 1; }
tail -1 gpurun_out/winc_inproc.log
# the saved library (ab_libs/libA.so) against this build: conv + wgrad shape sets
timeout -k 10 600 bash tools/ab_lib.sh ab_libs/libA.so detectron2_tensorflow_amd/lib/libd2mi_hip.so "kxk short_k wgrad" || exit 1
python3 - <<'PY'
import re, collections
cur = None; t = collections.defaultdict(lambda: collections.defaultdict(list)); sums = collections.defaultdict(set)
for l in open('gpurun_out/lib_ab.log'):
    if l.startswith('== LIB='): cur = l.split('=')[-1].strip(); continue
    m = re.match(r'(\S+)\s+([\d.]+) us.*sum (\S+)', l)
    if m and cur: t[m.group(1)][cur].append(float(m.group(2))); sums[m.group(1)].add(m.group(3))
tot = collections.Counter()
for shp, d in t.items():
    row = {k: min(v) for k, v in d.items()}
    for k, v in row.items(): tot[k] += v
    print(f"{shp:32s} " + "  ".join(f"{k}: {v:8.1f}" for k, v in row.items()))
print("TOTAL", dict(tot), "sums equal:", all(len(v) == 1 for v in sums.values()))
PY
for rep in 1 2; do for lib in ab_libs/libA.so detectron2_tensorflow_amd/lib/libd2mi_hip.so; do
  D2MI_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/libab_bench.log 2>&1 || { tail -5 gpurun_out/libab_bench.log; exit 1; }
  echo "$(basename $lib) $(tail -1 gpurun_out/libab_bench.log | cut -c1-160)"
done; done
