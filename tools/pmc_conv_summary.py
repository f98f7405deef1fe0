#!/usr/bin/env python
"""Average per-launch SQ counters of the conv kernels under gpurun_out/pmc_conv/."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_conv"
for d in sorted(glob.glob(os.path.join(root, "*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "conv_" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d), {k: f"{sum(v) / len(v):.3g}" for k, v in sorted(acc.items())})
