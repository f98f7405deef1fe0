#!/bin/bash
# GPU box: conv / wgrad parity tests on the current build, then an alternating
# A/B of a saved library (ab_libs/libA.so) against it on the conv shape sets,
# then the training step with each library twice (A B A B).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "conv or wgrad" > gpurun_out/libab_tests.log 2>&1 \
  || { tail -40 gpurun_out/libab_tests.log; exit 1; }
tail -1 gpurun_out/libab_tests.log
timeout -k 10 600 bash tools/ab_lib.sh ab_libs/libA.so detectron2_tensorflow_amd/lib/libd2mi_hip.so "kxk short_k" || exit 1
python3 - <<'PY'
import re, collections
cur = None; t = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open('gpurun_out/lib_ab.log'):
    if l.startswith('== LIB='): cur = l.split('=')[-1].strip(); continue
    m = re.match(r'(\S+)\s+([\d.]+) us', l)
    if m and cur: t[m.group(1)][cur].append(float(m.group(2)))
tot = collections.Counter()
for shp, d in t.items():
    row = {k: min(v) for k, v in d.items()}
    for k, v in row.items(): tot[k] += v
    print(f"{shp:32s} " + "  ".join(f"{k}: {v:8.1f}" for k, v in row.items()))
print("TOTAL", dict(tot))
PY
for rep in 1 2; do for lib in ab_libs/libA.so detectron2_tensorflow_amd/lib/libd2mi_hip.so; do
  D2MI_LIB=$lib timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/libab_bench.log 2>&1 || { tail -5 gpurun_out/libab_bench.log; exit 1; }
  echo "$(basename $lib) $(tail -1 gpurun_out/libab_bench.log | cut -c1-160)"
done; done
