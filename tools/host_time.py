#!/usr/bin/env python
"""Host enqueue time vs device time of bench.py's step.

Each step starts on an idle device: host_ms = time for step() to return
(Python + launches, plus any host syncs inside the step), wall_ms = time
until the device has finished it.  host_ms close to wall_ms means the step is
launch-bound, not kernel-bound.

usage: python tools/host_time.py [--mode train|infer] [--steps 5]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="train")
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    import bench
    sys.argv = [sys.argv[0], "--mode", a.mode]
    args = bench.parse()
    args.gpus = 1
    dev = torch.device("cuda", 0)
    from detectron2_tensorflow_amd import _C
    _C.load()
    cfg, model = bench.build(args, dev)
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
        hs, ws = [], []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            hs.append((t1 - t0) * 1e3)
            ws.append((t2 - t0) * 1e3)
    hs.sort()
    ws.sort()
    print(f"host_ms median {hs[len(hs) // 2]:.2f}  wall_ms median {ws[len(ws) // 2]:.2f}  "
          f"(min {hs[0]:.2f} / {ws[0]:.2f})")


if __name__ == "__main__":
    main()
