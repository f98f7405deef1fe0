#!/usr/bin/env python
"""cProfile of the host side of bench.py's training step (each step synced),
to find where the launch-bound host time goes.

usage: python tools/host_profile.py [--steps 3] [--top 40]
"""
import argparse
import cProfile
import os
import pstats
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    import bench
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    args.gpus = 1
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
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.steps):
        tr.step(batch)
        torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(a.top)
    st.sort_stats("cumulative").print_stats(a.top)


if __name__ == "__main__":
    main()
