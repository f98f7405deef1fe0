#!/usr/bin/env python
"""A/B of the NMS scans (tuning "nms_scan": 1 the fixed-point tile resolve,
0 the serial one) on RPN-shaped segments: 10 segments of 2,000 boxes, IoU
0.7, max_out 1,000 (and two other operating points).  Each arm's kept lists
must be identical; times are the whole ops.nms_segments call (keys, sort,
gather, mask, scan), interleaved rounds, median -- the difference is the scan.

    python tools/nms_scan_ab.py [--iters 50] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def boxes_like_rpn(rng, n, H=800, W=1333):
    c = rng.uniform([0, 0], [H, W], size=(n, 2))
    s = np.exp(rng.uniform(np.log(16), np.log(512), size=n))
    ar = np.exp(rng.uniform(np.log(0.5), np.log(2.0), size=n))
    h, w = s * np.sqrt(ar), s / np.sqrt(ar)
    b = np.stack([c[:, 0] - h / 2, c[:, 1] - w / 2, c[:, 0] + h / 2, c[:, 1] + w / 2], 1)
    return np.clip(b, 0, [H, W, H, W]).astype(np.float32)


def anchors_like_rpn(rng, n, stride=8, size=64, H=800, W=1333):
    """Unregressed proposals (a random-init RPN's): the anchor grid of one
    level -- 3 aspect ratios per position, neighbours overlapping above 0.7 --
    with a little jitter, the top-n of a random score."""
    ys, xs = np.meshgrid(np.arange(0, H, stride) + stride / 2, np.arange(0, W, stride) + stride / 2,
                         indexing="ij")
    c = np.stack([ys.ravel(), xs.ravel()], 1).repeat(3, 0)
    ar = np.tile([0.5, 1.0, 2.0], len(c) // 3)
    h, w = size * np.sqrt(ar), size / np.sqrt(ar)
    b = np.stack([c[:, 0] - h / 2, c[:, 1] - w / 2, c[:, 0] + h / 2, c[:, 1] + w / 2], 1)
    b = b + rng.normal(0, 0.5, size=b.shape)
    pick = rng.choice(len(b), size=n, replace=False)
    return np.clip(b[pick], 0, [H, W, H, W]).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.layers import ops
    _C.load()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    S, n = 10, 2000
    sc = torch.from_numpy(rng.normal(size=S * n).astype(np.float32)).to(dev)
    off = torch.arange(0, S * n + 1, n, dtype=torch.int32, device=dev)
    old = ops.get_tuning("nms_scan")
    rand = torch.from_numpy(np.concatenate([boxes_like_rpn(rng, n) for _ in range(S)])).to(dev)
    anch = torch.from_numpy(np.concatenate([anchors_like_rpn(rng, n, stride=4 << (i % 4), size=32 << (i % 4))
                                            for i in range(S)])).to(dev)
    for name, b, max_out, thr in (("random", rand, 1000, 0.7), ("random", rand, 2000, 0.7),
                                  ("random", rand, 100, 0.5), ("anchors", anch, 1000, 0.7),
                                  ("anchors", anch, 2000, 0.7)):
        res, times = {}, {0: [], 1: []}
        for arm in (1, 0):
            ops.set_tuning("nms_scan", arm)
            res[arm] = [t.cpu() for t in ops.nms_segments(b, sc, off, max_out, thr, seg_capacity=n)]
        same = all(torch.equal(x, y) for x, y in zip(res[0], res[1]))
        for _ in range(a.rounds):
            for arm in (1, 0):
                ops.set_tuning("nms_scan", arm)
                ops.nms_segments(b, sc, off, max_out, thr, seg_capacity=n)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    ops.nms_segments(b, sc, off, max_out, thr, seg_capacity=n)
                e1.record()
                torch.cuda.synchronize()
                times[arm].append(e0.elapsed_time(e1) * 1e3 / a.iters)
        kept = res[1][1].float().mean().item()
        print(f"{name:8s} max_out {max_out} thr {thr}: kept/segment {kept:.0f}  fixed-point "
              f"{statistics.median(times[1]):7.1f} us  serial {statistics.median(times[0]):7.1f} us  "
              f"identical {same}", flush=True)
    ops.set_tuning("nms_scan", old)


if __name__ == "__main__":
    main()
