#!/usr/bin/env python
"""Capture the graphed training step (engine/graphed.py) WITHOUT replaying
it and write every graph as a DOT file (hipGraphDebugDotPrint), then
summarise the node kinds: a diagnosis of what the captured graphs contain
(memcpy / memset nodes, host-memory operands, kernel names) that cannot
fault the GPU.

usage: python tools/graph_dump.py [--height 256 --width 320] [--out gpurun_out/graphs]
"""
import argparse
import collections
import glob
import os
import re
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def summarize(path):
    txt = open(path).read()
    kinds = collections.Counter()
    names = collections.Counter()
    for m in re.finditer(r'label="([^"]*)"', txt):
        lab = m.group(1)
        head = lab.split("\\n")[0].split("|")[0].strip("{} ")
        kinds[head[:40]] += 1
        k = re.search(r"(_Z\w+|Cijk\w+|\w*kernel\w*)", lab)
        if k:
            names[k.group(1)[:90]] += 1
    return txt, kinds, names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "graphs"))
    a = ap.parse_args()
    import bench
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.engine.graphed import GraphedTrainer
    sys.argv = [sys.argv[0], "--height", str(a.height), "--width", str(a.width)]
    args = bench.parse()
    args.gpus = 1
    dev = torch.device("cuda", 0)
    _C.load()
    cfg, model = bench.build(args, dev)
    batch = bench.synthetic_batch(args, dev, 0)
    bench.calibrate_scores(model, batch)
    tr = GraphedTrainer(cfg, model, experimental=True)
    tr.debug_dump_dir = a.out
    tr.step(batch)  # eager warm-up
    torch.cuda.synchronize()
    tr._on_stream(tr._capture_forward, batch)  # capture A and every B; no replay
    torch.cuda.synchronize()
    for f in sorted(glob.glob(os.path.join(a.out, "graph_*.dot"))):
        txt, kinds, names = summarize(f)
        print(f"== {os.path.basename(f)}: {len(txt)} bytes")
        print("  node label heads:", dict(kinds.most_common(12)))
        for n, c in names.most_common(80):
            print(f"  {c:4d}  {n}")
        for line in txt.splitlines():
            if re.search(r"(?i)memcpy|memset|host", line):
                print("  MEMCPY/MEMSET/HOST:", line[:300])


if __name__ == "__main__":
    main()
