#!/bin/bash
# FrozenBN fold kernel change check: the fold exactness tests, then the
# timed-region profile of the training bench (fold_bn_* time per step).
set -o pipefail
tag=${1:-fold}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "fold or train_step or whole" \
    --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
STEPS=10 bash tools/profile_bench.sh ${tag}
python3 - "$tag" <<'PY'
import csv, sys
for r in csv.DictReader(open(f"gpurun_out/{sys.argv[1]}_timed_kernel_stats.csv")):
    if "fold_bn" in r["Name"] or "sgd_" in r["Name"]:
        print(f"{float(r['TotalDurationNs']) / 10 / 1e3:8.1f} us/step  {r['Name'][:70]}")
PY
