#!/usr/bin/env python
"""Isolated time of the stem kernels at the bench geometry (2 x 800 x 1344):
d2mi_stem_conv and d2mi_stem_pool, events around --iters launches each."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    _C.load()
    dev = torch.device("cuda:0")
    x = torch.randn(2, 800, 1344, 3, device=dev) * 50
    w = torch.randn(7, 7, 3, 64, device=dev) / 147 ** 0.5
    w3 = ops.stem_conv_weights(w)
    y = ops.stem_conv(x, w3)
    shift = torch.randn(64, device=dev)
    for name, fn in (("stem_conv", lambda: ops.stem_conv(x, w3)),
                     ("stem_pool", lambda: ops.stem_pool(y, shift))):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name}: {e0.elapsed_time(e1) / a.iters * 1e3:.1f} us", flush=True)


if __name__ == "__main__":
    main()
