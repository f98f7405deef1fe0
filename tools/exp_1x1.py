#!/usr/bin/env python
"""1x1-conv (GEMM-shaped) timing: the MFMA conv kernel in split / f32 math,
with and without the fused residual, against torch.mm (hipBLASLt) and a plain
copy of the output size (HBM reference).

usage: python tools/exp_1x1.py [--shapes M,Cin,Cout;...]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402

SHAPES = "134400,64,256;8400,256,1024;33600,128,512;8400,1024,256;33600,512,128;134400,256,64"


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=SHAPES)
    a = ap.parse_args()
    _C.load()
    dev = torch.device("cuda:0")
    for sh in a.shapes.split(";"):
        M, Cin, Cout = map(int, sh.split(","))
        x = torch.randn(1, 1, M, Cin, device=dev)
        w = torch.randn(1, 1, Cin, Cout, device=dev) / Cin ** 0.5
        wp = ops.pack_conv_weights(w)
        r = torch.randn(1, 1, M, Cout, device=dev)
        y = torch.empty(1, 1, M, Cout, device=dev)
        fl = 2.0 * M * Cin * Cout
        res = {
            "split": timeit(lambda: ops.conv2d_nhwc(x, wp, None, 1, (0, 0), math_mode="split")),
            "split+r": timeit(lambda: ops.conv2d_nhwc(x, wp, None, 1, (0, 0), residual=r,
                                                      math_mode="split")),
            "f32": timeit(lambda: ops.conv2d_nhwc(x, wp, None, 1, (0, 0), math_mode="f32")),
            "mm": timeit(lambda: torch.mm(x.view(M, Cin), w.view(Cin, Cout))),
            "copy_out": timeit(lambda: y.copy_(r)),
        }
        mb = (M * Cin + M * Cout) * 4 / 1e6
        print(f"M={M} Cin={Cin} Cout={Cout} ({mb:.0f} MB in+out): " +
              "  ".join(f"{k} {v:.1f}us ({fl / v / 1e6:.0f} TF/s)" for k, v in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
