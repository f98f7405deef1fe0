#!/usr/bin/env python
"""Kernel statistics restricted to bench.py's timed region.

rocprofv3 --kernel-trace --marker-trace --output-format csv writes every
kernel of the run, including MIOpen's find-time benchmarking in the warmup.
bench.py brackets its timed K steps with the roctx range "timed_region"
(torch.cuda.nvtx -> roctx on ROCm); this keeps the kernels that START inside
that range and writes a stats CSV in rocprofv3's kernel_stats layout plus a
per-step summary, so the committed profile describes exactly what bench.py
timed.

usage: prof_window.py <rocprof out dir> <out stats csv> [--steps K]
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("out_csv")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--range", default="timed_region")
    a = ap.parse_args()
    kt = glob.glob(os.path.join(a.outdir, "**", "*kernel_trace.csv"), recursive=True)
    mt = glob.glob(os.path.join(a.outdir, "**", "*marker_api_trace.csv"), recursive=True)
    assert kt, "no kernel trace"
    lo, hi = None, None
    for f in mt:
        for r in csv.DictReader(open(f)):
            if r.get("Function", "") == a.range or r.get("Message", "") == a.range:
                lo, hi = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    assert lo is not None, "marker range %r not found" % a.range
    agg = collections.defaultdict(lambda: [0, 0, None, 0])
    first, last = None, None
    for f in kt:
        for r in csv.DictReader(open(f)):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if not (lo <= s <= hi):
                continue
            d = e - s
            g = agg[r["Kernel_Name"]]
            g[0] += 1
            g[1] += d
            g[2] = d if g[2] is None else min(g[2], d)
            g[3] = max(g[3], d)
            first = s if first is None else min(first, s)
            last = e if last is None else max(last, e)
    total = sum(v[1] for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    with open(a.out_csv, "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, (n, t, mn, mx) in rows:
            w.writerow([name, n, t, t / n, 100.0 * t / total, mn, mx])
    summ = {"range_ns": hi - lo, "kernel_busy_ns": total, "steps": a.steps,
            "range_ms_per_step": (hi - lo) / 1e6 / a.steps,
            "kernel_ms_per_step": total / 1e6 / a.steps,
            "kernels_per_step": sum(v[0] for v in agg.values()) / a.steps}
    with open(os.path.splitext(a.out_csv)[0] + "_summary.json", "w") as fo:
        json.dump(summ, fo, indent=1)
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
