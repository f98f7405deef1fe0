#!/usr/bin/env python
"""Per-shape time and TFLOP/s of the MFMA conv launches inside bench.py's step.

usage: python tools/conv_shapes.py [--mode train|infer] [--steps 3]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="train")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--no-handoff", action="store_true",
                    help="bottleneck residual-gradient hand-off off (A/B)")
    a = ap.parse_args()
    import bench
    sys.argv = [sys.argv[0], "--mode", a.mode]
    args = bench.parse()
    args.gpus = 1
    dev = torch.device("cuda", 0)
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.layers.ops import KernelTimer
    _C.load()
    cfg, model = bench.build(args, dev)
    if a.no_handoff:
        for m in model.modules():
            if hasattr(m, "grad_handoff"):
                m.grad_handoff = False
    batch = bench.synthetic_batch(args, dev, 0)
    bench.calibrate_scores(model, batch)
    if a.mode == "train":
        from detectron2_tensorflow_amd.engine import Trainer
        tr = Trainer(cfg, model)
        step = lambda: tr.step(batch)
        ctx = torch.enable_grad
    else:
        step = lambda: model.inference(batch)
        ctx = torch.no_grad
    with ctx():
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        KernelTimer.reset(enabled=True, detail=True)
        for _ in range(a.steps):
            step()
        KernelTimer.enabled = False
    rows = [(k, n, ms, w) for k, (n, ms, w) in KernelTimer.summary().items()
            if k.startswith("conv ") or k.startswith("wgrad ")]
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows)
    print(f"{'shape':48s} {'calls/step':>10s} {'ms/step':>8s} {'TF/s':>7s}")
    for k, n, ms, w in rows:
        print(f"{k:48s} {n / a.steps:10.1f} {ms / a.steps:8.3f} {w / ms / 1e9:7.1f}")
    print(f"total {tot / a.steps:.3f} ms/step")


if __name__ == "__main__":
    main()
