#!/usr/bin/env python
"""Graphed vs eager training steps side by side (engine/graphed.py), without
stopping at the first difference: per step the mask-row count each trainer
used, the loss values and every parameter / momentum tensor that differs
(max |diff|, count).  A diagnosis companion of tests/test_gpu_graphed.py.

usage: python tools/graph_diff.py [--steps 7] [--same-batch] [--eager-at 4]"""
import argparse
import os
import sys


import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=7)
    ap.add_argument("--same-batch", action="store_true")
    ap.add_argument("--eager-at", type=int, default=-1)
    a = ap.parse_args()
    from graph_audit import build
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.engine import Trainer
    from detectron2_tensorflow_amd.engine.graphed import GraphedTrainer
    from detectron2_tensorflow_amd.utils.synthetic import synthetic_train_batch
    torch.backends.cudnn.deterministic = True
    dev = torch.device("cuda", 0)
    _C.load()
    cfg, m_eager, b0 = build(dev, 256, 320)
    _, m_graph, _ = build(dev, 256, 320)
    m_graph.load_state_dict(m_eager.state_dict())
    b1 = synthetic_train_batch(2, 256, 320, 12, dev)
    b1["instances"]["is_valid"][:, 2:] = False
    batches = [b0] if a.same_batch else [b0, b1]
    eager = Trainer(cfg, m_eager)
    graphed = GraphedTrainer(cfg, m_graph, warmup=1, experimental=True)
    he, hg = eager.model.roi_heads, graphed.heads[0]
    names = [n for n, _ in m_eager.named_parameters()]
    for i in range(a.steps):
        b = batches[i % len(batches)]
        bg = {k: (v.clone() if torch.is_tensor(v) else {kk: vv.clone() for kk, vv in v.items()})
              for k, v in b.items()}
        torch.manual_seed(100 + i)
        le = eager.step(b)
        torch.manual_seed(100 + i)
        lg = graphed.eager_step(bg) if i == a.eager_at else graphed.step(bg)
        torch.cuda.synchronize()
        kind = ("eager warm-up" if i == 0 else "eager" if i == a.eager_at
                else f"replay {graphed.replays}")
        print(f"step {i} ({kind}): rows eager {he.last_mask_rows} graphed {hg.last_mask_rows}; "
              f"captured B: {sorted(graphed._B)}", flush=True)
        bad_l = [k for k in le if not torch.equal(le[k].reshape(()), lg[k].reshape(()))]
        print(f"  losses differing: {bad_l} "
              + " ".join(f"{k}={float(le[k]):.6g}/{float(lg[k]):.6g}" for k in bad_l), flush=True)
        nbad = 0
        for n, pe, pg in zip(names, m_eager.parameters(), m_graph.parameters()):
            if not torch.equal(pe, pg):
                d = (pe - pg).abs()
                nz = int((d > 0).sum())
                idx = torch.nonzero(d.reshape(-1) > 0).reshape(-1)
                print(f"  param {n} {tuple(pe.shape)}: {nz} differ, max {float(d.max()):.3g}, "
                      f"first flat index {int(idx[0])}, last {int(idx[-1])}", flush=True)
                nbad += 1
        pname = {id(p): n for n, p in m_eager.named_parameters()}
        mom = [pname[id(p)] for p in eager.optimizer.params]
        for n, ae, ag in zip(mom, eager.optimizer.accum, graphed.optimizer.accum):
            if not torch.equal(ae, ag):
                d = (ae - ag).abs()
                print(f"  momentum {n}: {int((d > 0).sum())} differ, max {float(d.max()):.3g}",
                      flush=True)
        print(f"  {nbad} parameters differ", flush=True)
    _C.raise_on_errors(dev)


if __name__ == "__main__":
    main()
