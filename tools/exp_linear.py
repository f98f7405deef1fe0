#!/usr/bin/env python
"""Box-head FC GEMMs (fwd / dgrad / wgrad) on the split-product MFMA conv
kernels vs hipBLASLt (torch f32), with the error of each against float64.

usage: python tools/exp_linear.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402

SHAPES = [(1024, 12544, 1024), (1024, 1024, 1024), (1024, 1024, 320), (1024, 1024, 84)]


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    _C.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    for M, K, N in SHAPES:
        x = torch.randn(M, K, generator=g).to(dev)
        w = (torch.randn(K, N, generator=g) / K ** 0.5).to(dev)
        gy = torch.randn(M, N, generator=g).to(dev)
        fl = 2.0 * M * K * N
        wp = ops.pack_conv_weights(w.view(1, 1, K, N))
        x4, gy4 = x.view(1, M, 1, K), gy.view(1, M, 1, N)
        runs = {
            "fwd_mfma": lambda: ops.conv2d_nhwc(x4, wp, None, 1, (0, 0)),
            "fwd_blas": lambda: x @ w,
            "dgrad_mfma": lambda: ops.conv2d_nhwc(gy4, w.view(1, 1, K, N), None, 1, (0, 0)),
            "dgrad_blas": lambda: gy @ w.t(),
            "wgrad_mfma": lambda: ops.conv2d_wgrad(x4, gy4, 1),
            "wgrad_blas": lambda: x.t() @ gy,
        }
        ref = {"fwd": x.double() @ w.double(), "dgrad": gy.double() @ w.double().t(),
               "wgrad": x.double().t() @ gy.double()}
        for name, fn in runs.items():
            us = timeit(fn, a.iters)
            out = fn().reshape(ref[name.split("_")[0]].shape).double()
            r = ref[name.split("_")[0]]
            err = ((out - r).abs().max() / r.abs().max()).item()
            print(f"M{M} K{K} N{N} {name:11s} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s  "
                  f"max_rel_err {err:.2e}", flush=True)


if __name__ == "__main__":
    main()
