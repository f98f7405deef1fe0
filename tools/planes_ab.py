"""Per-shape A/B of the warp-specialised conv's operand forms (run on the GPU
box): f32 rows split while staging (the default), pre-split weight planes
(w3), pre-split activation planes (x3), both -- interleaved rounds, median
us per launch; outputs must be bit-identical across the arms.  Also times the
split pass that makes the planes (d2mi_split_bf16x3) of x.

    python tools/planes_ab.py [--iters 20] [--rounds 3]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402

SHAPES = [  # N, H, W, Cin, Cout, k, form
    (2, 200, 336, 256, 256, 3, ""), (2, 200, 336, 256, 256, 3, "f"), (2, 100, 168, 256, 256, 3, ""),
    (2, 50, 84, 256, 256, 3, ""), (2, 50, 84, 256, 256, 3, "gf"), (2, 25, 42, 512, 512, 3, ""),
    (2, 100, 168, 128, 128, 3, ""), (2, 50, 84, 1024, 256, 1, ""), (2, 50, 84, 256, 1024, 1, "r"),
    (2, 25, 42, 2048, 512, 1, ""), (64, 14, 14, 256, 256, 3, ""),
]


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    _C.load()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    tot = {k: 0.0 for k in ("f32", "w3", "x3", "x3w3", "split_x")}
    for N, H, W, Cin, Cout, k, form in SHAPES:
        p = (k - 1) // 2
        x = torch.randn(N, H, W, Cin, device=dev, generator=g)
        w = torch.randn(k, k, Cin, Cout, device=dev, generator=g) / (k * k * Cin) ** 0.5
        wp = ops.pack_conv_weights(w)
        x3, w3 = ops.split_bf16x3(x), ops.split_bf16x3(wp)
        OH, OW = (H + 2 * p - k) + 1, (W + 2 * p - k) + 1
        res = torch.randn(N, OH, OW, Cout, device=dev, generator=g) if "r" in form else None
        gate = torch.randn(N, OH, OW, Cout, device=dev, generator=g) if "g" in form else None
        kw = dict(residual=res, relu_gate=gate, relu_after_add=(form == "r"), relu=(form == "r"),
                  flip_taps="f" in form, math_mode="split")
        arms = {"f32": {}, "w3": {"w3": w3}, "x3": {"x3": x3}, "x3w3": {"x3": x3, "w3": w3}}
        ys = {n: ops.conv2d_nhwc(x, wp, None, 1, (p, p), **kw, **extra) for n, extra in arms.items()}
        for n, y in ys.items():
            assert torch.equal(y, ys["f32"]), (n, float((y - ys["f32"]).abs().max()))
        t = {n: [] for n in list(arms) + ["split_x"]}
        for _ in range(a.rounds):
            for n, extra in arms.items():
                t[n].append(timeit(lambda: ops.conv2d_nhwc(x, wp, None, 1, (p, p), **kw, **extra),
                                   a.iters))
            t["split_x"].append(timeit(lambda: ops.split_bf16x3(x), a.iters))
        med = {n: statistics.median(v) for n, v in t.items()}
        fl = 2.0 * N * OH * OW * Cout * k * k * Cin
        for n in tot:
            tot[n] += med[n]
        print(f"{N}x{H}x{W}x{Cin}->{Cout} k{k} {form:2s} " + "  ".join(
            f"{n} {med[n]:7.1f}us" + (f" ({fl / med[n] / 1e6:5.1f} TF/s)" if n != "split_x" else "")
            for n in med), flush=True)
    print("total " + "  ".join(f"{n} {v:.1f}us" for n, v in tot.items()), flush=True)


if __name__ == "__main__":
    main()
