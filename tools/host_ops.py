#!/usr/bin/env python
"""Host (CPU) time of the training step by op and by autograd node
(torch.profiler, CPU activity only): which forward ops and which backward
nodes cost the host the most enqueue time.

usage: python tools/host_ops.py [--steps 3] [--top 40]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    import bench
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.engine import Trainer
    _C.load()
    cfg, model = bench.build(args, dev)
    batch = bench.synthetic_batch(args, dev, 0)
    bench.calibrate_scores(model, batch)
    tr = Trainer(cfg, model)
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        for _ in range(a.steps):
            tr.step(batch)
        torch.cuda.synchronize()
    ka = prof.key_averages()
    rows = sorted(ka, key=lambda e: -e.cpu_time_total)
    print(f"{'name':70s} {'calls/step':>10s} {'cpu_total_us/step':>18s} {'self_us/step':>13s}")
    for e in rows[:a.top]:
        print(f"{e.key[:70]:70s} {e.count / a.steps:10.1f} {e.cpu_time_total / a.steps:18.1f} "
              f"{e.self_cpu_time_total / a.steps:13.1f}")
    print("\nby self time:")
    for e in sorted(ka, key=lambda e: -e.self_cpu_time_total)[:a.top]:
        print(f"{e.key[:70]:70s} {e.count / a.steps:10.1f} {e.self_cpu_time_total / a.steps:13.1f}")


if __name__ == "__main__":
    main()
