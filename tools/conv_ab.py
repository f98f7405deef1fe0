#!/usr/bin/env python
"""Time a list of conv shapes (split-bf16 MFMA, the training step's forms) in
one process: for A/B runs of kernel knobs set through the environment.

    python tools/conv_ab.py [--iters 50] [--set res4]

Each shape: N,H,W,Cin,Cout,k,stride,form with form in
  plain | r (residual add + ReLU after) | g (ReLU gate: a dgrad epilogue) |
  gr (gate + residual) | w (the weight gradient, conv2d_wgrad, with bias).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402

SETS = {
    "short_k": ["2,200,336,64,256,1,1,r", "2,100,168,128,512,1,1,r", "2,50,84,256,1024,1,1,r",
                "2,25,42,512,2048,1,1,r", "2,50,84,256,1024,1,1,gr", "2,50,84,1024,256,1,1,g",
                "2,50,84,1024,256,1,1,plain", "2,100,168,512,128,1,1,g",
                "2,200,336,256,64,1,1,plain", "2,200,336,64,64,1,1,plain"],
    "wgrad": ["2,200,336,256,256,3,1,w", "2,100,168,256,256,3,1,w", "2,50,84,256,256,3,1,w",
              "2,100,168,128,128,3,1,w", "2,25,42,512,512,3,1,w", "32,14,14,256,256,3,1,w",
              "2,50,84,1024,256,1,1,w", "2,50,84,256,1024,1,1,w", "2,200,336,64,64,3,1,w"],
    # the res4 / res5 / p4-p6 shapes: few output tiles, split K
    "small_m": ["2,50,84,1024,256,1,1,plain", "2,50,84,1024,256,1,1,g", "2,50,84,256,1024,1,1,r",
                "2,50,84,256,1024,1,1,gr", "2,50,84,256,256,3,1,plain", "2,25,42,2048,512,1,1,plain",
                "2,25,42,2048,512,1,1,g", "2,25,42,512,2048,1,1,r", "2,25,42,512,512,3,1,plain",
                "2,25,42,256,256,3,1,plain", "2,13,21,256,256,3,1,plain",
                "2,50,84,256,1024,1,1,w", "2,50,84,1024,256,1,1,w", "2,25,42,512,512,3,1,w",
                "2,25,42,2048,512,1,1,w", "2,25,42,512,2048,1,1,w"],
    "kxk": ["2,200,336,256,256,3,1,plain", "2,50,84,256,256,3,1,plain",
            "2,100,168,128,128,3,1,plain", "2,25,42,512,512,3,1,plain",
            "2,200,336,64,64,3,1,plain", "32,14,14,256,256,3,1,plain"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--set", default="short_k")
    ap.add_argument("--shapes", default=None)
    a = ap.parse_args()
    shapes = a.shapes.split(";") if a.shapes else SETS[a.set]
    _C.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    for spec in shapes:
        parts = spec.split(",")
        N, H, W, Cin, Cout, k, s = map(int, parts[:7])
        form = parts[7]
        x = torch.randn(N, H, W, Cin, generator=g).to(dev)
        w = (torch.randn(k, k, Cin, Cout, generator=g) / (k * k * Cin) ** 0.5).to(dev)
        wp = ops.pack_conv_weights(w)
        p = (k - 1) // 2
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        if form == "w":
            dy = torch.randn(N, OH, OW, Cout, generator=g).to(dev)
            ref = ops.conv2d_wgrad(x, dy, k, s, (p, p), with_bias=True)[0]
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                y = ops.conv2d_wgrad(x, dy, k, s, (p, p), with_bias=True)[0]
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            fl = 2.0 * N * OH * OW * Cout * k * k * Cin
            print(f"{spec:32s} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s  "
                  f"sum {float(y.double().sum()):.6e}", flush=True)
            continue
        res = torch.randn(N, OH, OW, Cout, generator=g).to(dev) if "r" in form else None
        gate = torch.randn(N, OH, OW, Cout, generator=g).to(dev) if "g" in form else None
        kw = dict(residual=res, relu_gate=gate, relu_after_add=(form == "r"), relu=(form == "r"))
        ref = ops.conv2d_nhwc(x, wp, None, s, (p, p), math_mode="split", **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            y = ops.conv2d_nhwc(x, wp, None, s, (p, p), math_mode="split", **kw)
        e1.record()
        torch.cuda.synchronize()
        assert torch.equal(y, ref)
        us = e0.elapsed_time(e1) / a.iters * 1e3
        fl = 2.0 * N * OH * OW * Cout * k * k * Cin
        by = 4.0 * (N * H * W * Cin + N * OH * OW * Cout * (1 + (res is not None) + (gate is not None)))
        print(f"{spec:32s} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s {by / us / 1e3:7.0f} GB/s  "
              f"sum {float(y.double().sum()):.6e}", flush=True)


if __name__ == "__main__":
    main()
