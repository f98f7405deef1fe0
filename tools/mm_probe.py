#!/usr/bin/env python
"""hipBLASLt f32 GEMM (torch.mm, native f32 MFMA) against this repo's split
bf16x3 MFMA conv on the training step's 1x1 shapes (forward GEMM view:
pixels x Cin @ Cin x Cout), times as medians of interleaved rounds; and the
f32 GEMM's max relative difference to a float64 product next to the split
conv's."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402

SHAPES = [(8400, 1024, 256), (8400, 256, 1024), (2100, 2048, 512), (2100, 512, 2048),
          (33600, 512, 128), (33600, 128, 512), (8400, 1024, 512), (134400, 256, 64)]


def timeit(fn, iters):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    _C.load()
    dev = torch.device("cuda:0")
    torch.backends.cuda.matmul.allow_tf32 = False
    for M, K, N in SHAPES:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(K, N, device=dev) / K ** 0.5
        wp = ops.pack_conv_weights(w.reshape(1, 1, K, N))
        x4 = x.reshape(1, 1, M, K)
        t = {0: [], 1: []}
        for _ in range(a.rounds):
            t[0].append(timeit(lambda: torch.mm(x, w), a.iters))
            t[1].append(timeit(lambda: ops.conv2d_nhwc(x4, wp, None, 1, (0, 0), math_mode="split"),
                               a.iters))
        ref = (x.double() @ w.double())
        e_mm = ((torch.mm(x, w).double() - ref).abs().max() / ref.abs().max()).item()
        e_sp = ((ops.conv2d_nhwc(x4, wp, None, 1, (0, 0), math_mode="split").reshape(M, N).double()
                 - ref).abs().max() / ref.abs().max()).item()
        fl = 2.0 * M * K * N
        m0, m1 = statistics.median(t[0]), statistics.median(t[1])
        print(f"M {M:6d} K {K:5d} N {N:5d}: torch.mm {m0:7.1f} us ({fl / m0 / 1e6:6.1f} TF/s, "
              f"err {e_mm:.1e})  split conv {m1:7.1f} us ({fl / m1 / 1e6:6.1f} TF/s, err {e_sp:.1e})",
              flush=True)


if __name__ == "__main__":
    main()
