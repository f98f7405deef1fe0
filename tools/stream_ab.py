#!/usr/bin/env python
"""conv1x1_stream_kernel (tuning "conv_stream") against the tiled split conv
on the training step's stride-1 1x1 shapes and epilogue forms, in one
process: outputs compared bit for bit, times as medians of interleaved
rounds (each round: both arms, --iters launches each), and each launch's
bytes (every operand once + the output) as GB/s and a fraction of 8 TB/s.

    python tools/stream_ab.py [--iters 30] [--rounds 5] [--min-m 1]

Shapes: N,H,W,Cin,Cout,form with form in plain (bias) | relu | r (residual +
ReLU after) | g (ReLU gate) | gr (gate + residual)."""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402

SHAPES = [
    "2,200,336,64,256,r", "2,200,336,64,256,plain", "2,200,336,64,64,plain",
    "2,100,168,128,512,r", "2,100,168,128,512,gr", "2,100,168,128,128,plain",
    "2,50,84,256,1024,r", "2,50,84,256,1024,gr", "2,200,336,256,64,plain",
    "2,100,168,256,512,plain", "2,200,336,256,256,plain", "2,50,84,256,256,g",
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--min-m", type=int, default=-1,
                    help="conv_stream value of the stream arm (< 0: every eligible shape)")
    ap.add_argument("--shapes", default=None)
    ap.add_argument("--nt", type=int, default=None,
                    help="compare the stream kernel with conv_stream_nt 0 (arm 0) and this value")
    a = ap.parse_args()
    shapes = a.shapes.split(";") if a.shapes else SHAPES
    _C.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    tot = {0: 0.0, 1: 0.0}
    for spec in shapes:
        N, H, W, Cin, Cout = map(int, spec.split(",")[:5])
        form = spec.split(",")[5]
        x = torch.randn(N, H, W, Cin, generator=g).to(dev)
        w = (torch.randn(1, 1, Cin, Cout, generator=g) / Cin ** 0.5).to(dev)
        b = torch.randn(Cout, generator=g).to(dev) * 0.1
        wp = ops.pack_conv_weights(w)
        res = torch.randn(N, H, W, Cout, generator=g).to(dev) if "r" in form else None
        gate = torch.randn(N, H, W, Cout, generator=g).to(dev) if "g" in form else None
        kw = dict(residual=res, relu_gate=gate, relu_after_add=(form == "r"),
                  relu=(form in ("r", "relu")))
        run = lambda: ops.conv2d_nhwc(x, wp, b, 1, (0, 0), math_mode="split", **kw)  # noqa: E731
        outs, times = {}, {0: [], 1: []}
        def set_arm(arm):
            if a.nt is None:
                ops.set_tuning("conv_stream", a.min_m if arm else 0)
            else:
                ops.set_tuning("conv_stream", a.min_m)
                ops.set_tuning("conv_stream_nt", a.nt if arm else 0)
        for arm in (0, 1):
            set_arm(arm)
            outs[arm] = run()
        torch.cuda.synchronize()
        same = torch.equal(outs[0], outs[1])
        for _ in range(a.rounds):
            for arm in (0, 1):
                set_arm(arm)
                run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                e1.synchronize()
                times[arm].append(e0.elapsed_time(e1) / a.iters * 1e3)
        ops.set_tuning("conv_stream", 0)
        ops.set_tuning("conv_stream_nt", 0)
        med = {k: statistics.median(v) for k, v in times.items()}
        y = outs[0]
        byts = ops.conv_bytes(x, wp, y, b, None, res, gate)
        for k in med:
            tot[k] += med[k]
        print(f"{spec:26s} tiled {med[0]:7.1f} us ({byts / med[0] / 1e6 / 8:5.3f} of HBM)  "
              f"stream {med[1]:7.1f} us ({byts / med[1] / 1e6 / 8:5.3f})  "
              f"x{med[0] / med[1]:5.2f}  bit-identical {same}", flush=True)
    print(f"total tiled {tot[0]:.1f} us, stream {tot[1]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
