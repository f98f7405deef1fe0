#!/usr/bin/env python
"""Average FETCH_SIZE / WRITE_SIZE per dispatch of the hot kernels.

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch (rocprofv3).  gfx950
correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the
bytes of 16 B/lane coalesced reads, so it is doubled here; WRITE_SIZE is taken
as reported (exact for 16 B/lane stores; our conv epilogue stores 4 B/lane, an
uncalibrated width — noted in the output).

usage: pmc_summarize.py <fetch dir> <write dir> <out.json>
"""
import collections
import csv
import glob
import json
import os
import re
import sys

# (kernels of the group, the group's one-per-op kernel).  The split-K /
# partial reductions are counted with their group; per-launch figures divide
# by the op's main kernel count.  conv_mfma_kernel<WM, WN, TM, TN, DB, SPLIT,
# OCC, ML>: SPLIT (the sixth argument) tells the split-bf16 kernels from the
# f32 ones.  ROIAlign backward: its own roi_bwd_* kernels (the clear kernel, one
# per backward, is the main one: it writes the 183 MB of grad maps at
# 1333x800) PLUS anything dispatched between a roi_bwd_emit kernel and the
# next roi_bwd_runs kernel (r1/r2: the rocPRIM sort; since the r3 counting
# sort nothing), so `traffic` covers the same kernels as the HIP-event time of
# the backward.
SPLIT_CONV = r"conv_mfma_kernel<\d+, \d+, \d+, \d+, (?:true|false), true"
F32_CONV = r"conv_mfma_kernel<\d+, \d+, \d+, \d+, (?:true|false), false"
GROUPS = {
    "conv2d_split": (re.compile(SPLIT_CONV + r"|conv_ws_kernel|splitk_reduce\w*_kernel"),
                     re.compile(SPLIT_CONV + r"|conv_ws_kernel")),
    "conv2d_mfma": (re.compile(F32_CONV), None),
    "roi_align_fwd": (re.compile(r"roi_align_fwd_kernel<true"), None),  # split below
    "roi_align_bwd": (re.compile(r"roi_bwd_"), re.compile(r"roi_bwd_clear_kernel")),
    "conv_wgrad_split": (re.compile(r"conv_wgrad_split_kernel|conv_wgrad_ws_kernel|wgrad_reduce4?_kernel"),
                         re.compile(r"conv_wgrad_split_kernel|conv_wgrad_ws_kernel")),
    "conv_wgrad": (re.compile(r"conv_wgrad_kernel<"), None),
}
ROI_BWD_OPEN = re.compile(r"roi_bwd_emit_kernel")
ROI_BWD_CLOSE = re.compile(r"roi_bwd_runs_kernel")


def load(d, counter):
    """-> [(dispatch id, kernel name, grid size, value)] in dispatch order."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    disp = []
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            disp.append((int(r.get("Dispatch_Id", 0) or 0), r.get("Kernel_Name", ""),
                         int(float(r.get("Grid_Size", 0) or 0)), float(r["Counter_Value"])))
    disp.sort(key=lambda x: x[0])
    return disp


def members(disp, g, rx):
    """Dispatches of group g (the ROIAlign backward also takes its sort)."""
    out = []
    inside = False
    for d in disp:
        name = d[1]
        if g == "roi_align_bwd":
            if ROI_BWD_OPEN.search(name):
                inside = True
            elif ROI_BWD_CLOSE.search(name):
                inside = False
            if rx.search(name) or inside:
                out.append(d)
        elif rx.search(name):
            out.append(d)
    return out


def split_roi_fwd(disp):
    """The ROIAlign forward's box-pooler (7x7, ~1000 ROIs) and mask-pooler
    (14x14, a few dozen ROIs) launches, told apart by grid size: the box
    launches have the largest grids.  -> {"roi_align_fwd": [values],
    "roi_align_fwd_mask": [values]}"""
    rx = re.compile(r"roi_align_fwd_kernel<true")
    xs = [(g, v) for _, n, g, v in disp if rx.search(n)]
    if not xs:
        return {}
    gmax = max(g for g, _ in xs)
    return {"roi_align_fwd": [v for g, v in xs if g * 2 > gmax],
            "roi_align_fwd_mask": [v for g, v in xs if g * 2 <= gmax]}


def main():
    fd, wd, out = sys.argv[1:4]
    fdisp = load(fd, "FETCH_SIZE")
    wdisp = load(wd, "WRITE_SIZE")
    res = {"units": "bytes per dispatch", "fetch_correction": 2.0,
           "note": "FETCH_SIZE x2 (gfx950 16 B/lane reads); WRITE_SIZE as reported",
           "groups": {}}
    for g, (rx, main_rx) in GROUPS.items():
        main_rx = main_rx or rx
        fm, wm = members(fdisp, g, rx), members(wdisp, g, rx)
        if not fm and not wm:
            continue
        main_n = sum(1 for d in fm if main_rx.search(d[1]))
        fb, wb = sum(d[3] for d in fm), sum(d[3] for d in wm)
        res["groups"][g] = {
            "dispatches": len(fm), "main_kernel_dispatches": main_n,
            "fetch_bytes_per_launch": 2.0 * fb * 1024 / max(main_n, 1),
            "write_bytes_per_launch": wb * 1024 / max(main_n, 1),
        }
        res["groups"][g]["traffic_bytes_per_launch"] = (
            res["groups"][g]["fetch_bytes_per_launch"] + res["groups"][g]["write_bytes_per_launch"])
    # the ROIAlign forward per launch kind (grid size), replacing the average
    fs, ws = split_roi_fwd(fdisp), split_roi_fwd(wdisp)
    for g in fs:
        if fs[g]:
            fb, wb = 2.0 * sum(fs[g]) * 1024 / len(fs[g]), sum(ws.get(g, [])) * 1024 / max(len(ws.get(g, [])), 1)
            res["groups"][g] = {"dispatches": len(fs[g]), "main_kernel_dispatches": len(fs[g]),
                                "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                                "traffic_bytes_per_launch": fb + wb, "split_by": "grid size"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
