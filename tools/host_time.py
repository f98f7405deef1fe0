#!/usr/bin/env python
"""Host enqueue time vs device time of bench.py's step.

Each step starts on an idle device: host_ms = time for step() to return
(Python + launches, plus any host syncs inside the step), wall_ms = time
until the device has finished it.  blocked_in_syncs_ms = time the host sat
in the step's synchronising reads (utils/host_sync.py: the mask branch's
foreground count), waiting for the device to catch up; host_busy_ms =
host_ms - blocked: the host's own enqueue work.  host_busy close to wall_ms
means the step is launch-bound, not kernel-bound.

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
    ap.add_argument("--gc-off", action="store_true",
                    help="Python's cyclic garbage collector disabled for the timed steps")
    ap.add_argument("--cprofile", type=int, default=0,
                    help="also cProfile this many steps and print the top host functions")
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
    from detectron2_tensorflow_amd.utils import host_sync
    with ctx():
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        if a.gc_off:
            import gc
            gc.collect()
            gc.disable()
        hs, ws, bs = [], [], []
        for _ in range(a.steps):
            host_sync.reset()
            t0 = time.perf_counter()
            step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            hs.append((t1 - t0) * 1e3)
            ws.append((t2 - t0) * 1e3)
            bs.append(host_sync.blocked_s * 1e3)
        if a.cprofile:
            import cProfile
            import pstats
            pr = cProfile.Profile()
            # backward on this thread, so the profile sees the backward
            # functions (the autograd engine's device thread is invisible to it)
            with torch.autograd.set_multithreading_enabled(False):
                pr.enable()
                for _ in range(a.cprofile):
                    step()
                pr.disable()
            torch.cuda.synchronize()
            st = pstats.Stats(pr)
            st.sort_stats("tottime").print_stats(70)
            st.sort_stats("cumulative").print_stats(120)
    med = lambda v: sorted(v)[len(v) // 2]
    busy = [h - b for h, b in zip(hs, bs)]
    print(f"host_ms median {med(hs):.2f}  blocked_in_syncs_ms {med(bs):.2f}  "
          f"host_busy_ms {med(busy):.2f}  wall_ms median {med(ws):.2f}  "
          f"host_busy/wall {med(busy) / med(ws):.2f}")


if __name__ == "__main__":
    main()
