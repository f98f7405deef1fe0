#!/bin/bash
# ROIAlign-backward change check: its exactness tests, then the timed-region
# profile of the training bench (roi_bwd_* time per step).  usage: tools/roi_pass.sh <tag>
set -o pipefail
tag=${1:-roi}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -k "roi or deferred or train_step or whole" \
    --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
STEPS=10 bash tools/profile_bench.sh ${tag}
python3 - "$tag" <<'PY'
import csv, sys
tot = pix = 0.0
for r in csv.DictReader(open(f"gpurun_out/{sys.argv[1]}_timed_kernel_stats.csv")):
    if "roi_bwd" in r["Name"]:
        v = float(r["TotalDurationNs"]) / 10 / 1e3
        tot += v
        pix += v if "pixel" in r["Name"] else 0.0
print(f"roi_bwd us/step {tot:.1f}, pixel passes {pix:.1f}")
PY
