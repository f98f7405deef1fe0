#!/usr/bin/env python
"""Attribute GPU kernel time of bench.py's step to PyTorch ops (torch.profiler).

usage: python tools/torch_prof.py [--mode train|infer] [--steps 3] [--height 800 --width 1333]
Prints the top ops by self device time and writes gpurun_out/torch_prof_<mode>.txt.
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
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--width", type=int, default=1333)
    ap.add_argument("--rows", type=int, default=60)
    ap.add_argument("--stacks", action="store_true", help="group small ops by Python stack")
    a = ap.parse_args()
    import bench
    sys.argv = [sys.argv[0], "--mode", a.mode, "--height", str(a.height), "--width", str(a.width)]
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
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                     record_shapes=True, with_stack=a.stacks) as prof:
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
    table = prof.key_averages(group_by_input_shape=False).table(
        sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=60)
    shapes = prof.key_averages(group_by_input_shape=True).table(
        sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=50,
        max_shapes_column_width=90)
    if a.stacks:
        shapes = prof.key_averages(group_by_stack_n=6).table(
            sort_by="self_cuda_time_total", row_limit=a.rows, max_name_column_width=40)
    if a.stacks:
        # self device time of the small aten ops (the glue between the d2mi
        # kernels) by call site: the innermost package frame of the op's
        # Python stack, else its nearest autograd-node / Python-function
        # ancestor in the profiler's event tree
        agg = {}
        nstack = 0
        for e in prof.events():
            if not e.name.startswith("aten::") or e.self_device_time_total <= 0:
                continue
            site = None
            frames = [f for f in (e.stack or []) if "detectron2_tensorflow_amd" in f]
            if frames:
                nstack += 1
                site = frames[0].split("detectron2_tensorflow_amd/")[-1]
            par = e.cpu_parent
            while site is None and par is not None:
                n = par.name
                if ("Backward" in n or "evaluate_function" in n or ".py(" in n
                        or n.startswith("_")):
                    site = n[:90]
                par = par.cpu_parent
            k = (e.name, site or "?")
            t, c = agg.get(k, (0.0, 0))
            agg[k] = (t + e.self_device_time_total, c + 1)
        rows = sorted(agg.items(), key=lambda kv: -kv[1][0])[: a.rows]
        shapes = f"(events with a package stack: {nstack})\n" + "\n".join(
            f"{t / a.steps:9.1f} us/step {c / a.steps:6.1f} calls  {k[0]:28s} {k[1]}"
            for k, (t, c) in rows)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"torch_prof_{a.mode}.txt"), "w") as f:
        f.write(table + "\n\n" + shapes)
    print(table)


if __name__ == "__main__":
    main()
