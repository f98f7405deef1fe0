#!/usr/bin/env python
"""Per-kernel stats (calls, total / average / min / max ns, share) from a
rocprofv3 rocpd SQLite database (ROCm 7 writes results.db by default), in the
column layout of rocprofv3's kernel_stats.csv, optionally only kernels whose
name matches a regex.

usage: python tools/rocpd_stats.py <results.db> [--match REGEX] [--csv OUT]"""
import argparse
import collections
import csv
import re
import sqlite3
import sys


def stats(db, match=None):
    c = sqlite3.connect(db)
    names = dict(c.execute("select id, kernel_name from rocpd_info_kernel_symbol"))
    agg = collections.defaultdict(list)
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        agg[names.get(kid, str(kid))].append(e - s)
    total = sum(sum(v) for v in agg.values()) or 1
    rows = []
    for n, d in agg.items():
        if match and not re.search(match, n):
            continue
        rows.append((n, len(d), sum(d), sum(d) / len(d), 100.0 * sum(d) / total, min(d), max(d)))
    rows.sort(key=lambda r: -r[2])
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match")
    ap.add_argument("--csv")
    a = ap.parse_args()
    rows = stats(a.db, a.match)
    out = open(a.csv, "w", newline="") if a.csv else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in rows:
        w.writerow(r)


if __name__ == "__main__":
    main()
