"""Per-kernel timeline of ROIAlign backward sequences from a rocprofv3 kernel
trace: for the last few sequences (from the grad-map clear to the pixel pass)
print each kernel's start offset, duration and the gap before it.

    python tools/roi_bwd_timeline.py gpurun_out/prof_roi/<...>_kernel_trace.csv | <rocprofv3 -d dir>
"""
import csv
import glob
import os
import re
import sys


def main(path, last=4):
    if os.path.isdir(path):  # a rocprofv3 -d directory: its (first) kernel trace
        path = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seqs, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        if "roi_bwd_clear_kernel" in n and (cur is None or cur[-1][0].startswith("roi_bwd_pixel")):
            cur = []
            seqs.append(cur)
        if cur is not None:
            m = re.search(r"(roi_bwd_\w+|onesweep\w*|histogram\w*|__amd_rocclr_\w+|\w+_kernel)", n)
            short = m.group(1) if m else n[:40]
            cur.append((short, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
            if short.startswith("roi_bwd_pixel"):
                cur = None
    for s in seqs[-last:]:
        t0 = s[0][1]
        prev_end = t0
        print(f"--- sequence: {(s[-1][2] - t0) / 1e3:.1f} us first start to last end")
        for name, a, b in s:
            print(f"  +{(a - t0) / 1e3:7.1f} us  dur {(b - a) / 1e3:6.1f}  gap {(a - prev_end) / 1e3:6.1f}  {name[:70]}")
            prev_end = max(prev_end, b)


if __name__ == "__main__":
    main(sys.argv[1])
