#!/usr/bin/env python
"""Name the ops that put memset / memcpy nodes into the graphed training
step's captures (engine/graphed.py), WITHOUT replaying any graph.

After every aten op issued inside a capture the node census of the graph
being captured (d2mi_capture_census) is taken; an op whose census grew by a
memset or memcpy node is listed with its shapes (nodes from library calls
made through ctypes are counted against the next aten op).  At the end the
per-graph census GraphedTrainer took before instantiating each graph.

usage: python tools/graph_nodes.py [--height 256 --width 320]
"""
import argparse
import collections
import os
import sys

# the diagnosis needs captures that may still hold memset nodes: with the
# runtime's graph packet capture off GraphedTrainer accepts them
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=320)
    a = ap.parse_args()
    from graph_audit import build
    from torch.utils._python_dispatch import TorchDispatchMode
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.engine import graphed
    from detectron2_tensorflow_amd.utils import capture
    dev = torch.device("cuda", 0)
    _C.load()
    cfg, model, batch = build(dev, a.height, a.width)
    tr = graphed.GraphedTrainer(cfg, model, warmup=1)
    tr.step(batch)  # the eager warm-up step
    torch.cuda.synchronize()
    hits = collections.Counter()
    last = {}

    class NodeCensus(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            if capture.capturing():
                c = graphed.capture_census(dev) or {}
                for kind in ("memset", "memcpy"):
                    d = c.get(kind, 0) - last.get(kind, 0)
                    if d > 0:
                        shapes = [tuple(x.shape) for x in args if torch.is_tensor(x)][:3]
                        hits[(kind, str(func), str(shapes))] += d
                last.clear()
                last.update(c)
            return out

    real_finish = tr._finish

    def finish(g, name):
        last.clear()  # the next capture starts from an empty graph
        real_finish(g, name)

    tr._finish = finish
    with NodeCensus():
        tr._on_stream(tr._capture_forward, batch)  # A and every B[R]; nothing replayed
    torch.cuda.synchronize()
    print("ops that added memset / memcpy nodes (kind, op, first shapes): count", flush=True)
    for (kind, op, sh), c in sorted(hits.items(), key=lambda kv: (kv[0][0], -kv[1])):
        print(f"  {kind:7s} {c:5d}  {op}  {sh}", flush=True)
    print("per-graph node census (before instantiation):", flush=True)
    for name, c in tr.census.items():
        print(f"  {name:6s} {c}", flush=True)
    total = sum(c.get("memset", 0) for c in tr.census.values())
    print(f"memset nodes in all captures: {total}; graph packet capture "
          f"{'on' if graphed.packet_capture_on() else 'off'}", flush=True)


if __name__ == "__main__":
    main()
