#!/usr/bin/env python
"""In-process A/B of a Python-level switch on the training step: one trainer,
blocks of steps alternating between the arms (A B B A ...), each block timed
with a synchronize on both sides, so box-to-box and run-to-run drift cancels.

usage: python tools/ab_inproc.py --switch fpn_join [--blocks 8 --steps 10]
"""
import argparse
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _fpn_join(on):
    from detectron2_tensorflow_amd.modeling.necks.fpn import FPN
    FPN.JOIN_GRAD = on


def _pack_group(on):
    from detectron2_tensorflow_amd.layers.convolutional import PackGroup
    PackGroup.ENABLED = on


def _rpn_acc(on):
    from detectron2_tensorflow_amd.modeling.proposal_generator.rpn import _RPNHead1x1Fn
    _RPNHead1x1Fn.ACC_LEVELS = on


def _conv_ws(on):
    from detectron2_tensorflow_amd.layers import ops
    ops.set_tuning("conv_ws", 2 if on else 0)


def _wgrad_ws1(on):
    from detectron2_tensorflow_amd.layers import ops
    ops.set_tuning("wgrad_ws1", 6 if on else 0)


def _stem_mfma(on):
    from detectron2_tensorflow_amd.modeling.backbone.resnet import Stem
    Stem.MFMA_CONV = on


def _fused_sample(on):
    from detectron2_tensorflow_amd.modeling import matcher
    from detectron2_tensorflow_amd.modeling.roi_heads import roi_heads
    matcher.FUSED_SUBSAMPLE = on
    roi_heads.FUSED_ORDER = on


def _conv_epi(on):
    from detectron2_tensorflow_amd.layers import ops
    ops.set_tuning("conv_epi", 1 if on else 0)


def _rpn_conv_acc(on):
    from detectron2_tensorflow_amd.modeling.proposal_generator.rpn import StandardRPNHead
    StandardRPNHead.ACC_CONV_LEVELS = on


def _rpn_concat(on):
    from detectron2_tensorflow_amd.modeling.proposal_generator.rpn import StandardRPNHead
    StandardRPNHead.CONCAT_OUT = on


def _defer_pixels(on):
    from detectron2_tensorflow_amd.layers import ops
    ops.DEFER_PIXELS = on


def _gc_off(on):
    import gc
    if on:
        gc.disable()
    else:
        gc.enable()


def _mask_prep_early(on):
    from detectron2_tensorflow_amd.modeling.roi_heads.roi_heads import StandardROIHeads
    StandardROIHeads.MASK_PREP_EARLY = on


def _skinny_levels(on):
    from detectron2_tensorflow_amd.modeling.proposal_generator.rpn import _RPNHead1x1Fn
    _RPNHead1x1Fn.LEVELS_ONE_LAUNCH = on


SWITCHES = {"skinny_levels": _skinny_levels, "mask_prep_early": _mask_prep_early, "gc_off": _gc_off, "defer_pixels": _defer_pixels, "rpn_concat": _rpn_concat, "rpn_conv_acc": _rpn_conv_acc, "fpn_join": _fpn_join, "pack_group": _pack_group, "rpn_acc": _rpn_acc,
            "conv_ws": _conv_ws, "conv_epi": _conv_epi,
            "wgrad_ws1": _wgrad_ws1, "stem_mfma": _stem_mfma, "fused_sample": _fused_sample}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--switch", default="fpn_join",
                    help="one of %s, or tune:<key>[=on,off] (d2mi_set_tuning values, default 1,0)"
                    % ", ".join(sorted(SWITCHES)))
    ap.add_argument("--blocks", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--mode", default="train", help="train | infer (bench.py's modes)")
    ap.add_argument("--model", default=None, help="bench.py --model (default: its own)")
    a = ap.parse_args()
    import bench
    sys.argv = [sys.argv[0], "--mode", a.mode] + (["--model", a.model] if a.model else [])
    args = bench.parse()
    dev = torch.device("cuda", 0)
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.engine import Trainer
    _C.load()
    cfg, model = bench.build(args, dev)
    batch = bench.synthetic_batch(args, dev, 0)
    bench.calibrate_scores(model, batch)
    if a.mode == "train":
        tr = Trainer(cfg, model)
        run = lambda: tr.step(batch)  # noqa: E731
    else:
        torch.set_grad_enabled(False)
        fwd = model if bench.is_single_stage(model) else model.inference
        run = lambda: fwd(batch)  # noqa: E731
    if a.switch.startswith("tune:"):
        from detectron2_tensorflow_amd.layers import ops
        key, _, vals = a.switch[5:].partition("=")
        von, voff = (int(v) for v in (vals or "1,0").split(","))
        sw = lambda on: ops.set_tuning(key, von if on else voff)  # noqa: E731
    else:
        sw = SWITCHES[a.switch]
    for on in (True, False, True):
        sw(on)
        for _ in range(2):
            run()
    torch.cuda.synchronize()
    times = {True: [], False: []}
    for b in range(a.blocks):
        for on in ((True, False) if b % 2 == 0 else (False, True)):
            sw(on)
            run()  # one untimed step after the switch
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                run()
            torch.cuda.synchronize()
            times[on].append((time.perf_counter() - t0) * 1e3 / a.steps)
        print(f"block {b}: on {times[True][-1]:.3f} ms  off {times[False][-1]:.3f} ms", flush=True)
    mon, moff = statistics.median(times[True]), statistics.median(times[False])
    print(f"{a.switch}: on {mon:.3f} ms/step, off {moff:.3f} ms/step, on/off {mon / moff:.4f} "
          f"(medians over {a.blocks} blocks of {a.steps} steps)")


if __name__ == "__main__":
    main()
