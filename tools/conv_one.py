#!/usr/bin/env python
"""Run one conv shape repeatedly (for rocprofv3 PMC passes on the conv kernel).

    python tools/conv_one.py --shape 2,200,336,256,256,3,1 --mode split|f32 --iters 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="2,200,336,256,256,3,1")
    ap.add_argument("--mode", default="split")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    N, H, W, Cin, Cout, k, s = map(int, a.shape.split(","))
    _C.load()
    dev = torch.device("cuda:0")
    x = torch.randn(N, H, W, Cin, device=dev)
    w = torch.randn(k, k, Cin, Cout, device=dev) / (k * k * Cin) ** 0.5
    wp = ops.pack_conv_weights(w)
    p = (k - 1) // 2
    mm = "f32" if a.mode == "f32" else "split"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ops.conv2d_nhwc(x, wp, None, s, (p, p), math_mode=mm)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(a.iters):
        ops.conv2d_nhwc(x, wp, None, s, (p, p), math_mode=mm)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    fl = 2.0 * N * ((H + 2 * p - k) // s + 1) * ((W + 2 * p - k) // s + 1) * Cout * k * k * Cin
    print(f"{a.shape} {a.mode}: {ms * 1e3:.1f} us  {fl / ms / 1e9:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
