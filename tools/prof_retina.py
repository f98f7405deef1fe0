"""RetinaNet dense post-processing at 1333x800 (201,600 anchors x 80
classes per image = 16.1 M sigmoid scores) on synthetic head outputs:
cls logits ~ N(-3, 1) (BASELINE.md injection), deltas ~ N(0, 0.1^2).

    python tools/prof_retina.py [--iters 20] [--batch 2]

Prints one JSON line: us per call and the algorithmic GB/s of the logit scan
(4 B per score).  Run under rocprofv3 --kernel-trace --stats for the per-kernel
split."""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--width", type=int, default=1333)
    a = ap.parse_args()
    _C.load()
    dev = torch.device("cuda:0")
    N, A, K = a.batch, 9, 80
    H, W = -(-a.height // 32) * 32, -(-a.width // 32) * 32  # size_divisibility 32
    strides = [8, 16, 32, 64, 128]
    hw = [(math.ceil(H / s), math.ceil(W / s)) for s in strides]
    g = torch.Generator(device="cpu").manual_seed(0)
    cls = [(torch.randn(N, h, w, A * K, generator=g) - 3.0).to(dev) for h, w in hw]
    box = [(torch.randn(N, h, w, A * 4, generator=g) * 0.1).to(dev) for h, w in hw]
    cells = []
    for x in (32, 64, 128, 256, 512):
        sizes = [x, x * 2 ** (1 / 3), x * 2 ** (2 / 3)]
        rows = []
        for s in sizes:
            for r in (0.5, 1.0, 2.0):
                w_ = math.sqrt(s * s / r)
                h_ = r * w_
                rows.append([-h_ / 2, -w_ / 2, h_ / 2, w_ / 2])
        cells.append(torch.tensor(rows, dtype=torch.float32))

    def run():
        return ops.retinanet_inference(cls, box, strides, cells, K, 1000, 0.05, 0.5, 100)

    out = run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        out = run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    scores = sum(t.numel() for t in cls)
    print(json.dumps({"op": "retinanet_inference", "batch": N, "levels": hw, "scores": scores,
                      "us": round(ms * 1e3, 1), "alg_GBps": round(4 * scores / ms / 1e6, 1),
                      "detections": int(out[3].sum())}), flush=True)


if __name__ == "__main__":
    main()
