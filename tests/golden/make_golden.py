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

convert_d2_golden.npz: the reference's lib/convert_models/convert_d2.py
(convert_weights, convert_d2.py:4-187; it imports only numpy) applied to
seeded detectron2-named state dicts of five model layouts -- Mask R-CNN
R50-FPN (FrozenBN statistics, num_batches_tracked), RetinaNet R50 (P6P7,
4-conv towers, per-anchor box order), a Res5ROIHeads (C4) Mask R-CNN with
class-agnostic box regression, a Cascade R-CNN with a conv box head and GN
norms plus a deformable-conv offset, and a PanopticFPN semantic head.
Channel counts are shrunk (the conversion only transposes, renames and
permutes; the shapes that matter -- box-delta groups of 4, fc1's (C, h, w)
rows -- keep their structure).  Stored per case: the cfg fields the
conversion reads (JSON), every input array and every output array.

    python tests/golden/make_golden.py [/root/reference] [--only convert_d2]
"""
import json
import importlib.util
import os
import sys
import types

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "nms_golden.npz")
OUT_MC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "multiclass_nms_golden.npz")
OUT_BOX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "box_ops_golden.npz")
OUT_VOC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "voc_metrics_golden.npz")
OUT_D2 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "convert_d2_golden.npz")


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


class _NS:
    """A cfg-like attribute tree (the fields convert_weights reads)."""

    def __init__(self, d):
        for k, v in d.items():
            setattr(self, k, _NS(v) if isinstance(v, dict) else v)


def d2_state_dict(cfgd, rng):
    """A detectron2-named state dict for the layout cfgd describes (small,
    seeded values; the keys follow detectron2's module names)."""
    M = cfgd["MODEL"]
    d = {}
    C = 3  # shrunk channel count of every plain conv

    def arr(*shape):
        return rng.standard_normal(shape).astype(np.float32)

    def conv(name, o=C, i=C, k=1, norm="bn", bias=False, offset=False):
        d[name + ".weight"] = arr(o, i, k, k)
        if norm in ("bn", "bn_nbt"):
            d[name + ".norm.weight"] = arr(o)
            d[name + ".norm.bias"] = arr(o)
            d[name + ".norm.running_mean"] = arr(o)
            d[name + ".norm.running_var"] = np.abs(arr(o)) + 0.5
            if norm == "bn_nbt":
                d[name + ".norm.num_batches_tracked"] = np.array(7, np.int64)
        elif norm == "gn":
            d[name + ".norm.weight"] = arr(o)
            d[name + ".norm.bias"] = arr(o)
        if offset:
            d[name + "_offset.weight"] = arr(18, i, k, k)
            d[name + "_offset.bias"] = arr(18)
        if bias:
            d[name + ".bias"] = arr(o)

    def fc(name, o, i):
        d[name + ".weight"] = arr(o, i)
        d[name + ".bias"] = arr(o)

    fpn = M["NECK"]["NAME"] == "FPN"
    retina = M["NECK"]["TOP_BLOCK_TYPE"] == "P6P7"
    res5_head = M["ROI_HEADS"]["NAME"] == "Res5ROIHeads"
    bb = "backbone.bottom_up." if fpn else "backbone."
    conv(bb + "stem.conv1", k=7, norm="bn_nbt")
    blocks = {50: [3, 4, 6, 3], 101: [3, 4, 23, 3]}[M["RESNETS"]["DEPTH"]]
    for g in range(4):
        pre = "roi_heads." if (res5_head and g == 3 and not retina) else bb
        for b in range(blocks[g]):
            conv(f"{pre}res{g + 2}.{b}.conv1", norm="bn_nbt" if b % 2 else "bn")
            conv(f"{pre}res{g + 2}.{b}.conv2", k=3, norm="bn", offset=(g == 2 and b == 1 and
                                                                        M.get("_DEFORM", False)))
            conv(f"{pre}res{g + 2}.{b}.conv3")
            if b == 0:
                conv(f"{pre}res{g + 2}.{b}.shortcut")
    if retina:
        for lvl in (6, 7):
            conv(f"backbone.top_block.p{lvl}", k=3, norm=None, bias=True)
        lvls = (3, 4, 5)
    else:
        lvls = (2, 3, 4, 5) if fpn else ()
    for lvl in lvls:
        conv(f"backbone.fpn_lateral{lvl}", norm=None, bias=True)
        conv(f"backbone.fpn_output{lvl}", k=3, norm=None, bias=True)
    if retina:
        A = 9
        for i in range(M["RETINANET"]["NUM_CONVS"]):
            conv(f"head.cls_subnet.{2 * i}", k=3, norm=None, bias=True)
            conv(f"head.bbox_subnet.{2 * i}", k=3, norm=None, bias=True)
        conv("head.cls_score", o=A * 2, k=3, norm=None, bias=True)
        conv("head.bbox_pred", o=A * 4, k=3, norm=None, bias=True)
    elif M["META_ARCHITECTURE"] != "SemanticSegmentor":
        A = 3
        conv("proposal_generator.rpn_head.conv", k=3, norm=None, bias=True)
        conv("proposal_generator.rpn_head.objectness_logits", o=A, norm=None, bias=True)
        conv("proposal_generator.rpn_head.anchor_deltas", o=4 * A, norm=None, bias=True)
        h = M["ROI_BOX_HEAD"]
        K = 1 if h["CLS_AGNOSTIC_BBOX_REG"] else M["ROI_HEADS"]["NUM_CLASSES"]
        res = h["POOLER_RESOLUTION"]
        fc_in = M["NECK"]["OUT_CHANNELS"] if fpn else M["RESNETS"]["RES2_OUT_CHANNELS"] * 8
        if h["NUM_CONV"] > 0:
            fc_in = h["CONV_DIM"]
        fcd = h["FC_DIM"]
        stages = [f".{k}" for k in range(3)] if M["ROI_HEADS"]["NAME"] in (
            "CascadeROIHeads", "CascadeLCCHeads") else [""]
        for st in stages:
            for i in range(h["NUM_CONV"]):
                conv(f"roi_heads.box_head{st}.conv{i + 1}", o=h["CONV_DIM"], i=h["CONV_DIM"], k=3,
                     norm="gn")
            for i in range(h["NUM_FC"]):
                fc(f"roi_heads.box_head{st}.fc{i + 1}", fcd, fc_in * res * res if i == 0 else fcd)
            fc(f"roi_heads.box_predictor{st}.cls_score", M["ROI_HEADS"]["NUM_CLASSES"] + 1,
               fcd if h["NUM_FC"] else fc_in)
            fc(f"roi_heads.box_predictor{st}.bbox_pred", 4 * K, fcd if h["NUM_FC"] else fc_in)
        if M["MASK_ON"]:
            for i in range(M["ROI_MASK_HEAD"]["NUM_CONV"]):
                conv(f"roi_heads.mask_head.mask_fcn{i + 1}", k=3, norm=None, bias=True)
            conv("roi_heads.mask_head.deconv", k=2, norm=None, bias=True)
            conv("roi_heads.mask_head.predictor", o=M["ROI_HEADS"]["NUM_CLASSES"], norm=None,
                 bias=True)
    if M["META_ARCHITECTURE"] in ("PanopticFPN", "SemanticSegmentor"):
        ss = M["SEM_SEG_HEAD"]
        for i, feat in enumerate(ss["IN_FEATURES"]):
            for k in range(max(1, int(i + 2 - np.log2(ss["COMMON_STRIDE"])))):
                conv(f"sem_seg_head.{feat}.{2 * k}", k=3, norm="gn")
        conv("sem_seg_head.predictor", o=ss["NUM_CLASSES"], norm=None, bias=True)
    # detectron2 checkpoints carry the anchor generator's buffers too
    d["proposal_generator.anchor_generator.cell_anchors.0" if not retina
      else "anchor_generator.cell_anchors.0"] = arr(3, 4)
    return d


def d2_layouts():
    base = {"META_ARCHITECTURE": "GeneralizedRCNN", "MASK_ON": True,
            "NECK": {"NAME": "FPN", "TOP_BLOCK_TYPE": "LastLevelMaxPool", "OUT_CHANNELS": 3},
            "RESNETS": {"DEPTH": 50, "RES2_OUT_CHANNELS": 3},
            "ROI_HEADS": {"NAME": "StandardROIHeads", "NUM_CLASSES": 5},
            "ROI_BOX_HEAD": {"POOLER_RESOLUTION": 3, "NUM_CONV": 0, "CONV_DIM": 4, "NUM_FC": 2,
                             "FC_DIM": 6, "CLS_AGNOSTIC_BBOX_REG": False},
            "ROI_MASK_HEAD": {"NUM_CONV": 4},
            "RETINANET": {"NUM_CONVS": 4},
            "SEM_SEG_HEAD": {"IN_FEATURES": ["p2", "p3", "p4", "p5"], "COMMON_STRIDE": 4,
                             "NUM_CLASSES": 4}}

    def v(**over):
        m = json.loads(json.dumps(base))
        for path, val in over.items():
            node = m
            keys = path.split("__")
            for k in keys[:-1]:
                node = node[k]
            node[keys[-1]] = val
        return {"MODEL": m}

    return [
        ("mask_rcnn_R_50_FPN", v()),
        ("retinanet_R_50_FPN", v(META_ARCHITECTURE="RetinaNet", MASK_ON=False,
                                 NECK__TOP_BLOCK_TYPE="P6P7")),
        ("mask_rcnn_R_50_C4_agnostic", v(NECK__NAME="None", ROI_HEADS__NAME="Res5ROIHeads",
                                         ROI_BOX_HEAD__NUM_FC=0,
                                         ROI_BOX_HEAD__CLS_AGNOSTIC_BBOX_REG=True)),
        ("cascade_conv_head_gn_deform", v(MASK_ON=False, ROI_HEADS__NAME="CascadeROIHeads",
                                          ROI_BOX_HEAD__NUM_CONV=2,
                                          ROI_BOX_HEAD__CLS_AGNOSTIC_BBOX_REG=True, _DEFORM=True)),
        ("panoptic_fpn", v(META_ARCHITECTURE="PanopticFPN")),
    ]


def load_reference_convert_d2(ref_root):
    spec = importlib.util.spec_from_file_location(
        "_refconvert", os.path.join(ref_root, "lib", "convert_models", "convert_d2.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def convert_d2_cases(ref, rng):
    """{case}|cfg (JSON), {case}|in|<d2 name>, {case}|out|<reference name>."""
    data, names = {}, []
    for name, cfgd in d2_layouts():
        d = d2_state_dict(cfgd, rng)
        src = {k: v.copy() for k, v in d.items()}
        out = ref.convert_weights(d, _NS(cfgd))  # consumes d
        assert not d
        data[f"{name}|cfg"] = np.array(json.dumps(cfgd))
        for k, v in src.items():
            data[f"{name}|in|{k}"] = v
        for k, v in out.items():
            data[f"{name}|out|{k}"] = np.ascontiguousarray(v)
        names.append(name)
    data["cases"] = np.array(names)
    return data


def main(ref_root="/root/reference", *flags):
    if "--only" in flags and "convert_d2" in flags:
        d2 = convert_d2_cases(load_reference_convert_d2(ref_root), np.random.default_rng(20261019))
        np.savez_compressed(OUT_D2, **d2)
        print("wrote", OUT_D2, len(d2), "arrays")
        return
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
    d2 = convert_d2_cases(load_reference_convert_d2(ref_root), np.random.default_rng(20261019))
    np.savez_compressed(OUT_D2, **d2)
    print("wrote", OUT_D2, len(d2), "arrays")


if __name__ == "__main__":
    main(*sys.argv[1:])
