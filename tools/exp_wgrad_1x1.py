#!/usr/bin/env python
"""Small-pixel-count 1x1 weight gradients (res4 / res5 / FPN laterals): the
split-product MFMA wgrad kernel vs X^T.dY on hipBLASLt (torch.mm), per shape.

usage: python tools/exp_wgrad_1x1.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402

# (N, H, W, Cin, Cout, stride) of the conv input
SHAPES = [(2, 50, 84, 1024, 256, 1), (2, 50, 84, 256, 1024, 1), (2, 25, 42, 2048, 512, 1),
          (2, 25, 42, 512, 2048, 1), (2, 50, 84, 1024, 256, 1), (2, 100, 168, 512, 1024, 2),
          (2, 50, 84, 1024, 2048, 2), (2, 25, 42, 2048, 256, 1), (2, 50, 84, 1024, 512, 2)]


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    _C.load()
    dev = torch.device("cuda:0")
    for N, H, W, Cin, Cout, s in SHAPES:
        x = torch.randn(N, H, W, Cin, device=dev)
        OH, OW = (H - 1) // s + 1, (W - 1) // s + 1
        gy = torch.randn(N, OH, OW, Cout, device=dev)
        P = N * OH * OW
        fl = 2.0 * P * Cin * Cout

        def blas():
            xs = x if s == 1 else x[:, ::s, ::s]
            return torch.mm(xs.reshape(-1, Cin).t(), gy.reshape(-1, Cout))

        t_m = timeit(lambda: ops.conv2d_wgrad(x, gy, 1, s, (0, 0)))
        t_b = timeit(blas)
        ref = blas().double()
        got = ops.conv2d_wgrad(x, gy, 1, s, (0, 0)).reshape(Cin, Cout).double()
        err = float((got - ref).abs().max() / ref.abs().max())
        print(f"P={P} {Cin}->{Cout} s{s}: mfma {t_m:.1f}us ({fl / t_m / 1e6:.0f} TF/s)  "
              f"blas {t_b:.1f}us ({fl / t_b / 1e6:.0f} TF/s)  rel_err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
