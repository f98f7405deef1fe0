#!/usr/bin/env python
"""Which torch (non-d2mi) ops the training step still launches, with their
input shapes and the Python frames that issue them (torch.profiler), to pick
the next fusion.

usage: python tools/torch_ops_profile.py [--steps 2] [--ops add,copy_,...]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--by-count", action="store_true", help="order call sites by launches")
    ap.add_argument("--ops", default="aten::add,aten::add_,aten::copy_,aten::threshold_backward,"
                                      "aten::fill_,aten::zero_,aten::mul,aten::where,aten::cat")
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
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
        for _ in range(a.steps):
            tr.step(batch)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_input_shape=True)
    print(ka.table(sort_by="device_time_total", row_limit=a.top, max_name_column_width=40,
                   max_shapes_column_width=90))
    want = set(a.ops.split(","))
    # per-op call sites: the innermost frames inside this repository
    sites = {}
    for ev in prof.events():
        if ev.name not in want:
            continue
        frames = [f for f in (ev.stack or []) if "detectron2_tensorflow_amd" in f or "torch/autograd" in f]
        key = (ev.name, tuple(frames[:3]), str(ev.input_shapes)[:100])
        n, t = sites.get(key, (0, 0.0))
        sites[key] = (n + 1, t + ev.device_time_total)
    order = (lambda kv: -kv[1][0]) if a.by_count else (lambda kv: -kv[1][1])
    for (name, fr, shp), (n, t) in sorted(sites.items(), key=order)[:60]:
        print(f"{t / a.steps:9.1f}us {n // a.steps:4d} {name} {shp}")
        for f in fr:
            print("            ", f)


if __name__ == "__main__":
    main()
