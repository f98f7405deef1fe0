#!/usr/bin/env python
"""Audit the graphed training step's host-filled tables WITHOUT replaying any
graph (r5: the cause of the r4 hipGraph replay faults).

engine/graphed.py captures graph A (the forward) and one graph B[R] per
mask-branch row count into ONE private memory pool.  Some captured launches
read a small device table (the batched FrozenBN fold's entries, the fold
backward's, the fused Momentum-SGD's: device POINTERS) that the host fills
after the capture (utils/capture.py).  This tool records the caching
allocator's trace (torch.cuda.memory._record_memory_history) around every
capture and checks each table's bytes against every allocation made during a
capture window: an overlap means a captured kernel's temporary and the
host-written table share memory, so at replay that kernel overwrites the
table before the launch that reads it -- garbage pointers, an illegal
address.

  python tools/graph_audit.py --no-arena   # the r4 behaviour: tables from the pool
  python tools/graph_audit.py              # r5: tables in an arena reserved first

Exit status 1 if any table overlaps a captured allocation (--expect-clean)."""
import argparse
import os
import sys


import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CATS = {"num_thing_classes": 80, "num_stuff_classes": 53, "stuff_ignore_value": 0}
MARK = 7 << 20  # marker allocation sizes (multiples of 512 above 1 MiB: exact in the trace)


def build(dev, height, width):
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    from detectron2_tensorflow_amd.modeling import build_model
    from detectron2_tensorflow_amd.utils.synthetic import (calibrate_rcnn_scores,
                                                           synthetic_train_batch)
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, "configs", "COCO-InstanceSegmentation",
                                     "mask_rcnn_R_50_FPN_1x.yaml"))
    cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT = "raw"
    finalize(cfg, True, 1, CATS)
    torch.manual_seed(0)
    model = build_model(cfg).to(dev).train()
    batch = synthetic_train_batch(2, height, width, 11, dev)
    calibrate_rcnn_scores(model, batch)
    return cfg, model, batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--no-arena", action="store_true",
                    help="tables from the capture pool (the r4 code path)")
    ap.add_argument("--expect-clean", action="store_true")
    ap.add_argument("--ops", action="store_true",
                    help="also list the aten ops issued inside the captures (a census of the "
                         "ops that can put memset / memcpy nodes into the graphs)")
    a = ap.parse_args()
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.engine import graphed
    from detectron2_tensorflow_amd.utils import capture
    dev = torch.device("cuda", 0)
    _C.load()
    capture.ARENA = not a.no_arena
    cfg, model, batch = build(dev, a.height, a.width)
    tr = graphed.GraphedTrainer(cfg, model, warmup=1, experimental=True)
    tr.step(batch)  # the eager warm-up step
    torch.cuda.synchronize()

    # every torch.cuda.graph capture in engine/graphed.py bracketed by two
    # marker allocations (outside the capture) that the trace shows
    real_graph = torch.cuda.graph
    names = []

    class marked_graph:
        def __init__(self, *args, **kw):
            self.inner = real_graph(*args, **kw)

        def __enter__(self):
            k = len(names)
            names.append(f"capture{k}")
            t = torch.empty(MARK + 512 * 2 * k, dtype=torch.uint8, device=dev)
            del t
            return self.inner.__enter__()

        def __exit__(self, *exc):
            r = self.inner.__exit__(*exc)
            k = len(names) - 1
            t = torch.empty(MARK + 512 * (2 * k + 1), dtype=torch.uint8, device=dev)
            del t
            return r

    graphed.torch.cuda.graph = marked_graph
    capture.issued.clear()
    torch.cuda.memory._record_memory_history(enabled="all", context=None, stacks="python",
                                             max_entries=20_000_000)
    import collections
    from torch.utils._python_dispatch import TorchDispatchMode
    census = collections.Counter()

    class Census(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            if capture.capturing():
                shapes = [tuple(a.shape) for a in args if torch.is_tensor(a)][:2]
                census[(str(func), str(shapes))] += 1
            return func(*args, **(kwargs or {}))

    mode = Census() if a.ops else None
    try:
        # A and every B[R]: captured, tables flushed -- nothing replayed
        if mode is not None:
            with mode:
                tr._on_stream(tr._capture_forward, batch)
        else:
            tr._on_stream(tr._capture_forward, batch)
        torch.cuda.synchronize()
        snap = torch.cuda.memory._snapshot()
    finally:
        torch.cuda.memory._record_memory_history(enabled=None)
        graphed.torch.cuda.graph = real_graph
    trace = snap["device_traces"][dev.index]

    # capture windows from the markers; allocations made inside them
    opened, windows = {}, []
    allocs = []  # (trace index, addr, size, window)
    cur = None
    for i, e in enumerate(trace):
        act, size = e["action"], e.get("size", 0)
        if act == "alloc" and size >= MARK and (size - MARK) % 512 == 0 \
                and (size - MARK) // 512 < 2 * len(names):
            k, close = divmod((size - MARK) // 512, 2)
            if not close:
                opened[k] = i
                cur = k
            else:
                windows.append((k, opened.pop(k), i))
                cur = None
            continue
        if act == "alloc" and cur is not None:
            allocs.append((i, e["addr"], size, cur))
    print(f"graphs captured: {len(windows)} (A + {len(tr._B)} B[R]); allocations inside the "
          f"captures: {len(allocs)}; tables: {len(capture.issued)}", flush=True)
    label = {0: "A"}
    for j, r in enumerate(sorted(tr._B, key=lambda x: (x is None, x))):
        label[j + 1] = f"B[{r}]"

    bad = 0
    for addr, n, what in capture.issued:
        own = _own(allocs, addr)  # (a table taken from the pool: its own block, excluded)
        hits = [(i, aa, sz, w) for i, aa, sz, w in allocs
                if aa < addr + n and addr < aa + sz and i != own]
        where = sorted({label.get(w, w) for _, _, _, w in hits})
        if hits:
            bad += 1
        print(f"table {what:14s} @ {addr:#x} {n:6d} B: "
              f"{'OVERLAPS ' + str(len(hits)) + ' captured allocation(s) of ' + ', '.join(map(str, where)) if hits else 'no captured allocation overlaps it'}",
              flush=True)
    print(f"audit: {bad} of {len(capture.issued)} tables share memory with captured "
          f"temporaries ({'tables from the capture pool (r4)' if a.no_arena else 'table arena (r5)'})",
          flush=True)
    if a.ops:
        print("aten ops inside the captures (op, first shapes): count", flush=True)
        for (op, sh), c in sorted(census.items(), key=lambda kv: -kv[1]):
            print(f"  {c:5d}  {op}  {sh}", flush=True)
    if a.expect_clean and bad:
        sys.exit(1)


def _own(allocs, addr):
    """Trace index of the LAST allocation at exactly ``addr`` (a table taken
    from the pool: its own block)."""
    own = None
    for i, aa, _, _ in allocs:
        if aa == addr:
            own = i
    return own


if __name__ == "__main__":
    main()
