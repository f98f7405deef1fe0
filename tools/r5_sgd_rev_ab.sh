#!/bin/bash
# The SGD update's chunk order (tuning "sgd_rev"), twice each way: the two
# optimizer kernels' time from the timed-region kernel profile.
set -eo pipefail
for r in 0 1 0 1; do
  D2MI_SGD_REV=$r bash tools/profile_bench.sh sgdrev$r --steps 5 --warmup 3 > /dev/null
  python3 - "$r" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/sgdrev{sys.argv[1]}_timed_kernel_stats.csv")))
for r in rows:
    if "sgd_" in r["Name"]:
        print(f"sgd_rev={sys.argv[1]}  {float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:60]}")
PY
done
