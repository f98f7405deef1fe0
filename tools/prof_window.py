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
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("d2mi::(anonymous namespace)::", "").replace("void ", "")
    return name[:60]


def gaps(seq, path, steps):
    """Device-idle gaps between consecutive kernels of the window (one stream
    in practice): total per step, the kernels that start after the largest
    gaps (the GPU waited for the host to enqueue them), and the idle time
    summed over each kernel name that ends a gap."""
    seq.sort()
    idle, by_next, big = 0, collections.Counter(), []
    end = None
    for i, (s, e, n) in enumerate(seq):
        if end is not None and s > end:
            g = s - end
            idle += g
            by_next[short(n)] += g
            big.append((g, i, short(seq[i - 1][2]), short(n)))
        end = e if end is None else max(end, e)
    big.sort(reverse=True)
    per = max(1, len(seq) // max(1, steps))
    with open(path, "w") as fo:
        fo.write(f"idle between kernels: {idle / 1e6 / steps:.3f} ms/step over {steps} steps, "
                 f"{len(seq) / steps:.1f} kernels/step\n\nidle before kernel (ms/step):\n")
        for n, g in by_next.most_common(40):
            fo.write(f"{g / 1e6 / steps:8.3f}  {n}\n")
        fo.write("\nlargest gaps (us, index in step, previous -> next):\n")
        for g, i, p, n in big[:60]:
            fo.write(f"{g / 1e3:8.1f}  {i % per:4d}  {p} -> {n}\n")
        # idle per eighth of the step (where in the step the device starves)
        buckets = [0] * 8
        for g, i, _, _ in big:
            buckets[min(7, (i % per) * 8 // per)] += g
        fo.write("\nidle by eighth of the step's kernel sequence (ms/step): " +
                 " ".join(f"{b / 1e6 / steps:.2f}" for b in buckets) + "\n")
    return idle / 1e6 / steps


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
    seq = []
    for f in kt:
        for r in csv.DictReader(open(f)):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if not (lo <= s <= hi):
                continue
            d = e - s
            seq.append((s, e, r["Kernel_Name"]))
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
    summ["idle_ms_per_step"] = gaps(seq, os.path.splitext(a.out_csv)[0] + "_gaps.txt",
                                    a.steps)
    with open(os.path.splitext(a.out_csv)[0] + "_summary.json", "w") as fo:
        json.dump(summ, fo, indent=1)
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
