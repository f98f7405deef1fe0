#!/usr/bin/env python
"""RetinaNet inference post-processing (ops.retinanet_inference) at the C4
geometry -- 2 images of 800x1344 padded, 5 levels, A = 9, K = 80, logits
N(-3, 1) as bench.py's calibration, deltas N(0, 0.1^2) -- with the fused
four-launch pipeline (tuning "retina_fused" = 1) against the unfused one (0)
in one process: outputs compared exactly, times as medians of interleaved
rounds, and the fraction of HBM for the 129 MB of scores read once.

    python tools/retina_post_ab.py [--iters 20] [--rounds 5] [--dist normal]
    python tools/retina_post_ab.py --vars 0,1,2 --debug   # fused-path variants
                                    # (tuning "retina_var"; 4 = warm relaunches)
"""
import argparse
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402


def cell_anchors(size):
    out = []
    for s in (size, size * 2 ** (1 / 3), size * 2 ** (2 / 3)):
        for r in (0.5, 1.0, 2.0):
            h, w = s * np.sqrt(r), s / np.sqrt(r)
            out.append([-h / 2, -w / 2, h / 2, w / 2])
    return torch.tensor(out, dtype=torch.float32)


def orderable(x):
    """float32 tensor -> int64 keys whose order is the float order (common.h)."""
    u = x.contiguous().view(torch.int32).to(torch.int64) & 0xffffffff
    return torch.where(u >= 0x80000000, (~u) & 0xffffffff, u | 0x80000000)


def seg_debug(run, cls, N):
    """SegInfo {floor, exact_lo, k, exact, novf, pad, ts[10]} of every (image,
    level) segment, read from the head of the call's workspace, against the
    number of keys at or above the floor counted here; the wall-clock stamps
    (100 MHz) as phase durations and as offsets from the first kernel's start."""
    keep = []
    orig = _C.workspace
    _C.workspace = lambda nbytes, device: keep.append(orig(nbytes, device)) or keep[-1]
    old = ops.get_tuning("retina_fused")
    ops.set_tuning("retina_fused", 1)
    try:
        run()
        run()
    finally:
        _C.workspace = orig
        ops.set_tuning("retina_fused", old)
    torch.cuda.synchronize()
    L = len(cls)
    sz = 248  # sizeof(SegInfo)
    raw = keep[-1][:N * L * sz].cpu()
    i32 = raw.view(torch.int32).view(N * L, sz // 4)
    ts = raw.view(torch.int64).view(N * L, sz // 8)[:, 3:13]
    cy = raw.view(torch.int64).view(N * L, sz // 8)[:, 13:23]
    sub = raw.view(torch.int64).view(N * L, sz // 8)[:, 23:31]
    mhz = lambda a, b: (int(cy[s, b]) - int(cy[s, a])) / max(1, int(ts[s, b]) - int(ts[s, a])) * 100  # noqa
    t0 = int(ts[:, 0].min())
    us = lambda a, b: (int(b) - int(a)) / 100.0  # noqa: E731
    for s in range(N * L):
        n, l = divmod(s, L)
        f = int(i32[s, 0]) & 0xffffffff
        keys = orderable(cls[l][n].reshape(-1))
        r = ts[s]
        line = (f"seg {s} (image {n}, level {l}): len {keys.numel()} floor {f:#010x} k {int(i32[s, 2])} "
                f"exact {int(i32[s, 3])} novf {int(i32[s, 4])} ; "
                f"keys >= floor {int((keys >= f).sum())}"
                f" | floor {us(r[0], r[1]):.1f} us [{us(t0, r[0]):.1f}..{us(t0, r[1]):.1f}]"
                f" | finish at {us(t0, r[2]):.1f}: gather {us(r[2], r[3]):.1f} select {us(r[3], r[4]):.1f}"
                f" sort {us(r[4], r[5]):.1f} [keys {us(r[4], sub[s, 0]):.1f} kth {us(sub[s, 0], sub[s, 1]):.1f}"
                f" append {us(sub[s, 1], sub[s, 2]):.1f} bitonic({int(sub[s, 3])}) {us(sub[s, 2], r[5]):.1f}]"
                f" decode {us(r[5], r[6]):.1f} (end {us(t0, r[6]):.1f})"
                f" | clock MHz floor {mhz(0, 1):.0f} finish {mhz(2, 6):.0f}")
        if l == 0:
            line += (f" | nms at {us(t0, r[7]):.1f}: counts {us(r[7], r[8]):.1f} window {us(r[8], sub[s, 4]):.1f}"
                     f" scan({int(sub[s, 5])} tiles) {us(sub[s, 4], r[9]):.1f} [first tile"
                     f" {us(sub[s, 4], sub[s, 6]):.1f} rest {us(sub[s, 6], sub[s, 7]):.1f}"
                     f" outputs {us(sub[s, 7], r[9]):.1f}] first tile: rows"
                     f" {us(sub[s, 4], sub[s + 1, 4]):.1f} barrier {us(sub[s + 1, 4], sub[s + 1, 5]):.1f}"
                     f" resolve {us(sub[s + 1, 5], sub[s + 1, 6]):.1f}"
                     f" (end {us(t0, r[9]):.1f}) nms clock {mhz(7, 9):.0f} MHz")
        print(line, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--dist", default="normal", choices=["normal", "saturated"])
    ap.add_argument("--arms", default="0,1", help="retina_fused values to time")
    ap.add_argument("--vars", default="",
                    help="time the fused path under these tuning retina_var values instead")
    ap.add_argument("--from-model", action="store_true",
                    help="the head outputs of bench.py's calibrated RetinaNet R101-FPN on its "
                         "synthetic batch (the in-model score distribution) instead of iid logits")
    ap.add_argument("--debug", action="store_true",
                    help="print the fused path's per-segment floor state (workspace head)")
    a = ap.parse_args()
    _C.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    N, A, K = 2, 9, 80
    hw = [(100, 168), (50, 84), (25, 42), (13, 21), (7, 11)]
    strides = [8, 16, 32, 64, 128]
    cls, box = [], []
    if a.from_model:
        import bench
        sys.argv = [sys.argv[0], "--model", "retinanet_R_101_FPN", "--mode", "infer"]
        bargs = bench.parse()
        _, model = bench.build(bargs, dev)
        batch = bench.synthetic_batch(bargs, dev, 0)
        bench.calibrate_scores(model, batch)
        with torch.no_grad():
            det = model.detector
            feats = model.neck(model.backbone(model.preprocess_image(batch).tensor))
            c_out, b_out = det.head([feats[f] for f in det.in_features])
        cls = [t.contiguous() for t in c_out]
        box = [t.contiguous() for t in b_out]
        N = cls[0].shape[0]
        print("from model: levels", [tuple(t.shape) for t in cls], flush=True)
    for h, w in ([] if a.from_model else hw):
        x = torch.randn(N, h, w, A * K, generator=g) - 3.0
        if a.dist == "saturated":
            x = torch.where(torch.rand(x.shape, generator=g) < 0.2, x + 30.0, x)
        cls.append(x.to(dev))
        box.append((torch.randn(N, h, w, A * 4, generator=g) * 0.1).to(dev))
    cells = [cell_anchors(s) for s in (32, 64, 128, 256, 512)]
    nbytes = 4 * sum(t.numel() for t in cls)
    run = lambda: ops.retinanet_inference(cls, box, strides, cells, K, 1000, 0.05, 0.5, 100)  # noqa
    key = "retina_var" if a.vars else "retina_fused"
    arms = [int(v) for v in (a.vars or a.arms).split(",")]
    if a.debug:
        for arm in (arms if a.vars else [0]):
            if a.vars:
                print(f"-- retina_var={arm}", flush=True)
                ops.set_tuning("retina_var", arm)
            seg_debug(run, cls, N)
        if a.vars:
            ops.set_tuning("retina_var", 0)
        arms = [v for v in arms if not v & 4]  # (relaunch arms: stamps only)
    old = ops.get_tuning(key)
    if a.vars:
        ops.set_tuning("retina_fused", 1)
    outs = {}
    for arm in arms:
        ops.set_tuning(key, arm)
        outs[arm] = [t.clone() for t in run()]
    torch.cuda.synchronize()
    ref = outs[arms[0]]
    for arm in arms[1:]:
        same = all(torch.equal(x, y) for x, y in zip(ref, outs[arm]))
        print(f"{key}={arm} outputs equal to {key}={arms[0]}: {same} "
              f"(valid {int(outs[arm][3].sum())} vs {int(ref[3].sum())})", flush=True)
    times = {arm: [] for arm in arms}
    for _ in range(a.rounds):
        for arm in arms:
            ops.set_tuning(key, arm)
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            e1.synchronize()
            times[arm].append(e0.elapsed_time(e1) / a.iters * 1e3)
    ops.set_tuning(key, old)
    for arm in arms:
        m = statistics.median(times[arm])
        print(f"{key}={arm}: {m:8.1f} us per call  ({nbytes / m / 1e6 / 8:.3f} of HBM for "
              f"{nbytes / 1e6:.1f} MB of scores)  rounds {[round(v, 1) for v in times[arm]]}",
              flush=True)


if __name__ == "__main__":
    main()
