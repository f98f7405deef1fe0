"""Generates tests/golden/nms_golden.npz from the REFERENCE's own numpy NMS,
and tests/golden/box_ops_golden.npz from its numpy IoU, clip and decode.

Runs only in the build container (needs /root/reference): loads
lib/structures/np_box_list.py, np_box_ops.py and np_box_list_ops.py by file
path under a synthetic package (bypassing lib/structures/__init__.py, which
imports TensorFlow) and records, for seeded inputs, the indices kept by
np_box_list_ops.non_max_suppression (np_box_list_ops.py:146-217).

That numpy NMS matches TF's NonMaxSuppressionV3 only on inputs that avoid its
documented differences (float64 intersection, no min/max corner normalisation,
no area<=0 rule, argsort tie order), so the generator draws positive-area,
tie-free inputs and rejects sets with any pairwise IoU within 1e-4 of the
threshold.  The committed .npz is data (inputs + expected outputs); no
reference source travels with it.

box_ops_golden.npz (same loader):
  * np_box_ops.iou (np_box_ops.py:48-63: intersection in float64 through
    np.zeros, float32 areas) of two seeded box sets -> float64 IoU matrix;
    the sets avoid near-ties (each GT's best IoU, and each overlapped box's
    best GT, leads the runner-up by > 1e-4) and IoUs within 1e-4 of the
    matcher thresholds 0.3 / 0.5 / 0.7;
  * np_box_list_ops.clip_to_window (np_box_list_ops.py:319-350: fmin / fmax,
    then the boxes with area > 0 kept) -> clipped boxes + kept indices;
  * np_box_ops.apply_box_deltas (np_box_ops.py:85-113: weights (1, 1, 1, 1),
    ymax = ymin + h) -> decoded boxes, |dh|, |dw| below Box2BoxTransform's
    clamp log(1000/16) so the two formulas differ only by rounding.

multiclass_nms_golden.npz (same loader):
  * np_box_list_ops.multi_class_non_max_suppression (np_box_list_ops.py:220-290:
    per class, score > thresh, NMS, then every class's survivors sorted by
    score) on 300 clustered boxes x 12 classes whose scores are the softmax
    (float32, TF's exp(x - max) * (1 / sum)) of seeded logits; the class-offset
    NMS of fast_rcnn_inference (fast_rcnn.py:141-145) makes the same per-class
    decisions on these inputs: boxes inside [0, 900) with max_coord + 1
    offsets separate the classes, every pairwise IoU is 1e-4 away from the
    threshold, candidate scores are 2e-6 apart and 1e-5 away from score_thresh, and
    the survivors (< 100) fit topk_per_image.  Stored: boxes, logits, the
    selected boxes / scores / classes and each one's ROI row (matched back by
    exact box equality: the reference's BoxList drops extra fields).

voc_metrics_golden.npz: the reference's lib/evaluation/metrics.py
(compute_precision_recall / compute_average_precision, metrics.py:7-95) on
seeded detections: tie-free scores, bool and weighted-float labels, a class
with no detections; the file uses np.float / np.bool / np.NAN, which numpy 2
removed, so those aliases (float, bool, nan) are restored before it loads.

    python tests/golden/make_golden.py [/root/reference]
"""
import importlib.util
import os
import sys
import types

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "nms_golden.npz")
OUT_MC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "multiclass_nms_golden.npz")
OUT_BOX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "box_ops_golden.npz")
OUT_VOC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "voc_metrics_golden.npz")


def load_reference_metrics(ref_root):
    for name, v in (("float", float), ("bool", bool), ("NAN", np.nan)):
        if name not in np.__dict__:
            setattr(np, name, v)
    spec = importlib.util.spec_from_file_location(
        "_refmetrics", os.path.join(ref_root, "lib", "evaluation", "metrics.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def voc_metrics_cases(metrics, rng):
    data, n = {}, 0
    for size, frac, weighted, extra_gt in [(50, 0.4, False, 5), (400, 0.2, False, 30),
                                           (1000, 0.6, True, 100), (7, 0.5, False, 0),
                                           (0, 0.0, False, 12)]:
        scores = (rng.permutation(size) + rng.uniform(0.1, 0.9, size)) / max(size, 1)
        labels = rng.uniform(size=size) < frac
        if weighted:
            labels = labels * rng.uniform(0.5, 1.0, size)
        num_gt = int(np.ceil(np.sum(labels))) + extra_gt
        prec, rec = metrics.compute_precision_recall(scores, labels, num_gt)
        ap = metrics.compute_average_precision(prec, rec)
        data.update({f"v{n}_scores": scores, f"v{n}_labels": labels,
                     f"v{n}_num_gt": np.array(num_gt), f"v{n}_precision": prec,
                     f"v{n}_recall": rec, f"v{n}_ap": np.array(ap)})
        n += 1
    data["num_cases"] = np.array(n)
    return data


def load_reference_np_ops(ref_root):
    sdir = os.path.join(ref_root, "lib", "structures")
    pkg = types.ModuleType("_refstruct")
    pkg.__path__ = [sdir]
    sys.modules["_refstruct"] = pkg
    mods = {}
    for name in ["np_box_list", "np_box_ops", "np_box_list_ops"]:
        spec = importlib.util.spec_from_file_location(f"_refstruct.{name}",
                                                      os.path.join(sdir, name + ".py"))
        m = importlib.util.module_from_spec(spec)
        sys.modules[f"_refstruct.{name}"] = m
        spec.loader.exec_module(m)
        setattr(pkg, name, m)
        mods[name] = m
    return mods


def random_boxes(rng, n, extent=800.0, min_side=4.0, max_side=200.0, clusters=None):
    if clusters:
        centers = rng.uniform(0, extent, size=(clusters, 2))
        c = centers[rng.integers(0, clusters, size=n)] + rng.normal(0, 12, size=(n, 2))
    else:
        c = rng.uniform(0, extent, size=(n, 2))
    hw = np.exp(rng.uniform(np.log(min_side), np.log(max_side), size=(n, 2)))
    b = np.concatenate([c - hw / 2, c + hw / 2], axis=1)
    return b.astype(np.float32)


def iou64(b):
    b = b.astype(np.float64)
    a = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    ih = np.clip(np.minimum(b[:, None, 2], b[None, :, 2]) - np.maximum(b[:, None, 0], b[None, :, 0]), 0, None)
    iw = np.clip(np.minimum(b[:, None, 3], b[None, :, 3]) - np.maximum(b[:, None, 1], b[None, :, 1]), 0, None)
    inter = ih * iw
    return inter / (a[:, None] + a[None, :] - inter)


def make_case(rng, mods, n, thr, max_out, clusters):
    for _ in range(100):
        boxes = random_boxes(rng, n, clusters=clusters)
        iou = iou64(boxes)
        np.fill_diagonal(iou, 0)
        if np.any(np.abs(iou - thr) < 1e-4):
            continue
        scores = rng.permutation(n).astype(np.float32) / np.float32(n) + np.float32(0.001)
        bl = mods["np_box_list"].BoxList(boxes.copy())
        bl.add_field("scores", scores.copy())
        bl.add_field("idx", np.arange(n))
        res = mods["np_box_list_ops"].non_max_suppression(bl, max_output_size=max_out,
                                                          iou_threshold=thr,
                                                          score_threshold=-np.inf)
        keep = res.get_field("idx").astype(np.int32)
        return boxes, scores, keep
    raise RuntimeError("could not draw a threshold-safe case")


def box_ops_cases(mods, rng):
    ops, lops, bl = mods["np_box_ops"], mods["np_box_list_ops"], mods["np_box_list"]
    data = {}
    for _ in range(200):
        gt = random_boxes(rng, 20, extent=600.0, min_side=16.0, max_side=300.0)
        anchors = random_boxes(rng, 3000, extent=600.0, min_side=8.0, max_side=300.0,
                               clusters=60)
        # many anchors close to the GT so every matcher label occurs
        near = gt[rng.integers(0, 20, size=1000)] + rng.normal(0, 6, size=(1000, 4)).astype(np.float32)
        anchors[:1000] = np.concatenate([np.minimum(near[:, :2], near[:, 2:] - 2),
                                         np.maximum(near[:, 2:], near[:, :2] + 2)], 1)
        iou = ops.iou(gt.astype(np.float32), anchors.astype(np.float32))
        srt = np.sort(iou, axis=0)
        if np.any((srt[-1] > 0) & (srt[-1] - srt[-2] < 1e-4)):
            continue
        srt_g = np.sort(iou, axis=1)
        if np.any(srt_g[:, -1] - srt_g[:, -2] < 1e-4):
            continue
        if any(np.any(np.abs(iou - t) < 1e-4) for t in (0.3, 0.5, 0.7)):
            continue
        data.update(iou_gt=gt, iou_boxes=anchors, iou=iou)
        break
    else:
        raise RuntimeError("could not draw a tie-free IoU case")
    boxes = random_boxes(rng, 500, extent=900.0, min_side=4.0, max_side=400.0) - np.float32(100)
    window = np.array([0, 0, 640, 853], np.float32)
    blist = bl.BoxList(boxes.copy())
    blist.add_field("idx", np.arange(500))
    clipped = lops.clip_to_window(blist, window)
    data.update(clip_boxes=boxes, clip_window=window, clip_out=clipped.get().astype(np.float32),
                clip_keep=clipped.get_field("idx").astype(np.int32))
    dboxes = random_boxes(rng, 2000, extent=1333.0, min_side=4.0, max_side=800.0)
    deltas = rng.normal(0, 0.5, size=(2000, 4)).astype(np.float32)
    deltas[:, 2:] = np.clip(deltas[:, 2:], -4.0, 4.0)
    data.update(dec_boxes=dboxes, dec_deltas=deltas,
                dec_out=ops.apply_box_deltas(dboxes.copy(), deltas.copy()).astype(np.float32))
    return data


def softmax_tf32(logits):
    """float32 softmax in TF's CPU order: e = exp(x - max), e * (1 / sum(e))."""
    x = logits.astype(np.float32)
    e = np.exp(x - x.max(axis=1, keepdims=True)).astype(np.float32)
    return (e * (np.float32(1) / e.sum(axis=1, keepdims=True, dtype=np.float32))).astype(np.float32)


def multiclass_case(mods, rng, R=120, K=6, thr=0.5, score_thresh=0.3):
    lops, bl = mods["np_box_list_ops"], mods["np_box_list"]
    for _ in range(500):
        boxes = np.clip(random_boxes(rng, R, extent=800.0, min_side=40.0, max_side=70.0,
                                     clusters=6), 1.0, 899.0).astype(np.float32)
        boxes[:, 2:] = np.maximum(boxes[:, 2:], boxes[:, :2] + 4.0)
        iou = iou64(boxes)
        np.fill_diagonal(iou, 0)
        if np.any(np.abs(iou - thr) < 1e-4):
            continue
        logits = rng.normal(0, 2.0, size=(R, K + 1)).astype(np.float32)
        probs = softmax_tf32(logits)
        sc = probs[:, :K]
        cand = np.sort(sc[sc > score_thresh])
        if len(cand) == 0 or np.any(np.diff(cand) < 2e-6) or \
                np.any(np.abs(sc - score_thresh) < 1e-5):
            continue
        blist = bl.BoxList(boxes.copy())
        blist.add_field("scores", sc.copy())
        res = lops.multi_class_non_max_suppression(blist, score_thresh, thr, 100)
        sel = res.get()
        if not 20 <= len(sel) < 100 or len(sel) >= len(cand):
            continue  # want suppression to happen and every survivor to fit
        rows = np.array([np.nonzero((boxes == b).all(1))[0][0] for b in sel], np.int32)
        return dict(mc_boxes=boxes, mc_logits=logits, mc_sel_boxes=sel.astype(np.float32),
                    mc_sel_scores=res.get_field("scores").astype(np.float32),
                    mc_sel_classes=res.get_field("classes").astype(np.int64),
                    mc_sel_rows=rows, mc_params=np.array([thr, score_thresh], np.float64))
    raise RuntimeError("could not draw a threshold-safe multi-class case")


def main(ref_root="/root/reference"):
    mods = load_reference_np_ops(ref_root)
    rng = np.random.default_rng(20261015)
    cases = [
        (64, 0.5, 64, None), (64, 0.3, 10, 4), (300, 0.7, 1000, 20), (1000, 0.7, 1000, 60),
        (1000, 0.5, 100, 30), (2000, 0.7, 1000, 100), (2000, 0.5, 300, 40), (5, 0.5, 5, None),
    ]
    data = {}
    for i, (n, thr, max_out, clusters) in enumerate(cases):
        b, s, k = make_case(rng, mods, n, thr, max_out, clusters)
        data[f"c{i}_boxes"] = b
        data[f"c{i}_scores"] = s
        data[f"c{i}_keep"] = k
        data[f"c{i}_params"] = np.array([thr, max_out], np.float64)
    data["num_cases"] = np.array(len(cases))
    np.savez_compressed(OUT, **data)
    print("wrote", OUT, {k: v.shape for k, v in data.items() if k.endswith("_keep")})
    box = box_ops_cases(mods, np.random.default_rng(20261016))
    np.savez_compressed(OUT_BOX, **box)
    print("wrote", OUT_BOX, {k: v.shape for k, v in box.items()})
    mc = multiclass_case(mods, np.random.default_rng(20261017))
    np.savez_compressed(OUT_MC, **mc)
    print("wrote", OUT_MC, {k: v.shape for k, v in mc.items()})
    voc = voc_metrics_cases(load_reference_metrics(ref_root), np.random.default_rng(20261018))
    np.savez_compressed(OUT_VOC, **voc)
    print("wrote", OUT_VOC, {k: v.shape for k, v in voc.items()})


if __name__ == "__main__":
    main(*sys.argv[1:])
