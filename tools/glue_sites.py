#!/usr/bin/env python
"""Count the aten ops of one training step by Python call site (the innermost
frame in this package) with a TorchDispatchMode: the small torch ops between
the d2mi kernels (each a ~4-6 us launch).  Forward and the Python parts of
custom backwards (the engine runs them on this thread's mode stack only when
it propagates it; counts cover what it sees).

    python tools/glue_sites.py [--rows 60]
"""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = os.path.join(ROOT, "detectron2_tensorflow_amd")

SKIP = {"aten.view.default", "aten._unsafe_view.default", "aten.detach.default",
        "aten.t.default", "aten.as_strided.default", "aten.slice.Tensor", "aten.select.int",
        "aten.unsqueeze.default", "aten.squeeze.dim", "aten.permute.default",
        "aten.expand.default", "aten.reshape.default", "aten.alias.default",
        "aten.empty.memory_format", "aten.empty_strided.default", "aten.split.Tensor",
        "aten.unbind.int", "aten.transpose.int", "aten._reshape_alias.default",
        "aten.lift_fresh.default", "aten.is_same_size.default", "aten.unsqueeze_.default",
        "aten.sym_size.int", "aten.sym_stride.int", "aten.sym_numel.default",
        "aten.squeeze.default", "aten.chunk.default", "aten.narrow.default",
        "aten.split_with_sizes.default", "aten.empty_like.default", "aten.new_empty.default"}


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.count = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if name not in SKIP:
            site = "?"
            for fr in reversed(traceback.extract_stack(limit=40)):
                if fr.filename.startswith(PKG) or fr.filename.endswith("bench.py"):
                    site = f"{os.path.relpath(fr.filename, ROOT)}:{fr.lineno} {fr.name}"
                    break
            self.count[(name, site)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=60)
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
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    mode = Sites()
    with mode:
        tr.step(batch)
    torch.cuda.synchronize()
    tot = sum(mode.count.values())
    print(f"{tot} aten ops (views and allocations excluded)")
    by_site = collections.Counter()
    for (n, s), c in mode.count.items():
        by_site[s] += c
    print("--- by site")
    for s, c in by_site.most_common(a.rows):
        ops = ", ".join(f"{n.split('.')[1]}x{k}" for (n, s2), k in mode.count.most_common()
                        if s2 == s)[:150]
        print(f"{c:5d}  {s:70s} {ops}")


if __name__ == "__main__":
    main()
