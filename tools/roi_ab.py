#!/usr/bin/env python
"""In-process A/B of the ROIAlign forward variants (d2mi_set_tuning
"roi_fwd" bits, csrc/roi_align.hip) on the training step's OWN inputs: one
bench.py training step runs with ops.roi_align wrapped to capture the box
pooler's call (p2..p5 maps, the 1,024 sampled ROIs) and the mask pooler's;
each arm's output must be bit-identical to arm 0's; the arms are timed in
interleaved rounds (median).  Unique-bytes model as bench.py's roofline.

    python tools/roi_ab.py [--arms 0,1,2,4,8,15] [--iters 50] [--rounds 5]
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="0,1,2,4,8,15")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--key", default="roi_fwd")
    a = ap.parse_args()
    arms = [int(v) for v in a.arms.split(",")]
    import bench
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.engine import Trainer
    from detectron2_tensorflow_amd.layers import ops
    lib = _C.load()
    cfg, model = bench.build(args, dev)
    batch = bench.synthetic_batch(args, dev, 0)
    bench.calibrate_scores(model, batch)
    tr = Trainer(cfg, model)
    for _ in range(2):
        tr.step(batch)
    calls = []
    orig = ops.roi_align

    def spy(features, boxes, box_ind, output_size, scales, *rest, **kw):
        calls.append(([f.detach() for f in features], boxes.detach().clone(),
                      box_ind.detach().clone(), output_size, scales, rest,
                      {k: v for k, v in kw.items() if k != "grad_share"}))
        return orig(features, boxes, box_ind, output_size, scales, *rest, **kw)

    ops.roi_align = spy
    try:
        tr.step(batch)
    finally:
        ops.roi_align = orig
    torch.cuda.synchronize()
    for feats, boxes, bi, osz, scales, rest, kw in calls:
        if feats[0].shape[-1] < 64:
            continue
        run = lambda: orig(feats, boxes, bi, osz, scales, *rest, **kw)
        outs, times = {}, {v: [] for v in arms}
        for v in arms:
            ops.set_tuning(a.key, v)
            outs[v] = run()
        torch.cuda.synchronize()
        same = {v: bool(torch.equal(outs[v], outs[arms[0]])) for v in arms[1:]}
        for _ in range(a.rounds):
            for v in arms:
                ops.set_tuning(a.key, v)
                run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.iters * 1e3)
        R = boxes.shape[0]
        oh = osz if isinstance(osz, int) else osz[0]
        C = feats[0].shape[-1]
        o = outs[arms[0]]
        print(f"R={R} out={oh}x{oh} levels={len(feats)} identical={same}", flush=True)
        for v in arms:
            t = sorted(times[v])[len(times[v]) // 2]
            print(f"  {a.key}={v:3d}: {t:7.2f} us  out {o.numel() * 4 / t / 1e3:7.1f} GB/s",
                  flush=True)
    ops.set_tuning(a.key, -1)  # the default variant


if __name__ == "__main__":
    main()
