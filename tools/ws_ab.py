#!/usr/bin/env python
"""In-process A/B of the conv kernel-selection knob d2mi_set_tuning(key, v)
over the training step's conv shapes: every arm's output must be
bit-identical to arm 0's, and each arm is timed in interleaved rounds (the
median per shape is printed, then the total).

    python tools/ws_ab.py [--key ws] [--arms 0,2,3] [--set all] [--iters 20] [--rounds 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_ab import SETS  # noqa: E402
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--key", default="conv_ws")
    ap.add_argument("--arms", default="0,2,3")
    ap.add_argument("--set", default="all")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default=None, help="';'-separated N,H,W,Cin,Cout,k,s,form")
    a = ap.parse_args()
    arms = [int(v) for v in a.arms.split(",")]
    names = list(SETS) if a.set == "all" else a.set.split(",")
    wg = a.key.startswith("wgrad")
    shapes = ([s for n in names for s in SETS[n] if s.endswith(",w") == wg] if a.shapes is None
              else a.shapes.split(";"))
    lib = _C.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    tot = {v: 0.0 for v in arms}
    flops_tot = 0.0
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
            run = lambda: torch.cat([t.reshape(-1) for t in ops.conv2d_wgrad(
                x, dy, k, s, (p, p), with_bias=True)])
        else:
            res = torch.randn(N, OH, OW, Cout, generator=g).to(dev) if "r" in form else None
            gate = torch.randn(N, OH, OW, Cout, generator=g).to(dev) if "g" in form else None
            kw = dict(residual=res, relu_gate=gate, relu_after_add=(form == "r"), relu=(form == "r"))
            run = lambda: ops.conv2d_nhwc(x, wp, None, s, (p, p), math_mode="split", **kw)
        outs, times = {}, {v: [] for v in arms}
        for v in arms:
            ops.set_tuning(a.key, v)
            outs[v] = run()
        torch.cuda.synchronize()
        same = {v: bool(torch.equal(outs[v], outs[arms[0]])) for v in arms[1:]}
        for _ in range(a.rounds):
            for v in arms:
                ops.set_tuning(a.key, v)
                run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.iters * 1e3)
        fl = 2.0 * N * OH * OW * Cout * k * k * Cin
        flops_tot += fl
        med = {v: sorted(t)[len(t) // 2] for v, t in times.items()}
        for v in arms:
            tot[v] += med[v]
        cols = "  ".join(f"{a.key}={v}: {med[v]:8.1f} us {fl / med[v] / 1e6:6.1f} TF/s"
                         for v in arms)
        print(f"{spec:30s} {cols}  identical={same}", flush=True)
    ops.set_tuning(a.key, arms[0])
    print("TOTAL " + "  ".join(f"{a.key}={v}: {tot[v]:9.1f} us ({flops_tot / tot[v] / 1e6:6.1f} TF/s)"
                               for v in arms), flush=True)


if __name__ == "__main__":
    main()
