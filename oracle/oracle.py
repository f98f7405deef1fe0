"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of the reference's detection hot path, following the
reference Python glue line by line (file:line cited per function) and calling
the plain-C restatement of the TF 1.15 CPU kernels in ``ref_ops.c`` for the
kernels themselves (CropAndResize, NonMaxSuppressionV3, TopKV2 and the
Box2BoxTransform decode).  float32 everywhere, step by step, no fused ops.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this module, and only as the checker / the timed CPU baseline.

Parity status: NMS and IoU are pinned against the reference's own numpy NMS
(lib/structures/np_box_list_ops.py:146-217) through committed golden vectors;
everything else is pinned by hand-computed known answers (tests/test_oracle.py)
— the reference has no tests or fixtures and its TF kernels cannot run here.
"""
import ctypes
import math
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "ref_ops.c")
LIB = os.path.join(HERE, "build", "liboracle.so")

F32 = np.float32
EPS = F32(sys.float_info.epsilon)  # poolers.py:37
LN2 = F32(math.log(2))             # poolers.py:42
DEFAULT_SCALE_CLAMP = F32(math.log(1000.0 / 16))  # box_regression.py:10


def build(force=False):
    """Compile ref_ops.c with gcc (no FMA contraction, OpenMP over boxes/segments)."""
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        cmd = ["gcc", "-O2", "-fPIC", "-shared", "-std=c11", "-ffp-contract=off",
               "-fno-fast-math", "-fopenmp", SRC, "-o", LIB, "-lm"]
        subprocess.run(cmd, check=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _f32(a):
    return np.ascontiguousarray(a, dtype=F32)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


# ----------------------------------------------------------------- kernels
def crop_and_resize_tf(image, boxes, box_ind, crop_size):
    """tf.image.crop_and_resize (bilinear, extrapolation 0) on normalised boxes."""
    image, boxes, box_ind = _f32(image), _f32(boxes).reshape(-1, 4), _i32(box_ind)
    N, H, W, C = image.shape
    R = boxes.shape[0]
    ch, cw = crop_size
    out = np.empty((R, ch, cw, C), F32)
    rc = lib().oracle_crop_and_resize(_p(image), N, H, W, C, _p(boxes), _p(box_ind), R, ch, cw,
                                      _p(out))
    if rc != 0:
        raise ValueError("box_ind has values outside [0, batch_size)")
    return out


def crop_and_resize_grad_image(grads, boxes, box_ind, image_shape):
    grads, boxes, box_ind = _f32(grads), _f32(boxes).reshape(-1, 4), _i32(box_ind)
    R, ch, cw, C = grads.shape
    N, H, W = image_shape
    out = np.zeros((N, H, W, C), F32)
    fn = lib().oracle_crop_and_resize_grad_image
    rc = fn(_p(grads), _p(boxes), _p(box_ind), R, ch, cw, N, H, W, C, _p(out))
    if rc != 0:
        raise ValueError("box_ind has values outside [0, batch_size)")
    return out


def roi_align(image, boxes, box_ind, output_size, spatial_scale, sampling_ratio, aligned=True,
              pad_border=True):
    """ROIAlign.call (lib/layers/roi_align.py:45-66) -> crop_and_resize wrapper
    (lib/layers/functional.py:100-166) on one feature level."""
    image, boxes, box_ind = _f32(image), _f32(boxes).reshape(-1, 4), _i32(box_ind)
    N, H, W, C = image.shape
    R = boxes.shape[0]
    oh, ow = output_size
    out = np.empty((R, oh, ow, C), F32)
    fn = lib().oracle_roi_align_level
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                   ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    rc = fn(_p(image), N, H, W, C, _p(boxes), _p(box_ind), R, oh, ow, float(F32(spatial_scale)),
            int(sampling_ratio), int(bool(aligned)), int(bool(pad_border)), _p(out))
    if rc != 0:
        raise ValueError("box_ind has values outside [0, batch_size)")
    return out


def nms(boxes, scores, max_output_size, iou_threshold=0.5, score_threshold=-np.inf):
    """tf.image.non_max_suppression (NonMaxSuppressionV3)."""
    if not 0.0 <= iou_threshold <= 1.0:
        raise ValueError("iou_threshold must be in [0, 1]")
    if max_output_size < 0:
        raise ValueError("max_output_size must be non-negative")
    boxes, scores = _f32(boxes).reshape(-1, 4), _f32(scores).reshape(-1)
    out = np.empty(max(int(max_output_size), 1), np.int32)
    fn = lib().oracle_nms
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                   ctypes.c_float, ctypes.c_void_p]
    n = fn(_p(boxes), _p(scores), boxes.shape[0], int(max_output_size), float(iou_threshold),
           float(score_threshold), _p(out))
    return out[:n].copy()


def nms_batched(boxes, scores, offsets, max_out, iou_threshold):
    boxes, scores, offsets = _f32(boxes).reshape(-1, 4), _f32(scores), _i32(offsets)
    S = offsets.shape[0] - 1
    keep = np.empty((S, max(max_out, 1)), np.int32)
    num = np.empty(S, np.int32)
    fn = lib().oracle_nms_batched
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                   ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]
    fn(_p(boxes), _p(scores), _p(offsets), S, int(max_out), float(iou_threshold), _p(keep),
       _p(num))
    return keep[:, :max_out], num


def top_k(values, k):
    """tf.nn.top_k(sorted=True): value desc, ties lowest index first."""
    values = _f32(values).reshape(-1)
    k = min(int(k), values.shape[0])
    vals = np.empty(max(k, 1), F32)
    idx = np.empty(max(k, 1), np.int32)
    lib().oracle_topk(_p(values), values.shape[0], k, _p(vals), _p(idx))
    return vals[:k].copy(), idx[:k].copy()


def apply_deltas(deltas, boxes, weights, scale_clamp=DEFAULT_SCALE_CLAMP):
    """Box2BoxTransform.apply_deltas (lib/modeling/box_regression.py:76-123)."""
    deltas, boxes = _f32(deltas), _f32(boxes).reshape(-1, 4)
    N = boxes.shape[0]
    K = deltas.shape[1] // 4 if deltas.ndim == 2 else 1
    deltas = deltas.reshape(N, K * 4)
    out = np.empty_like(deltas)
    fn = lib().oracle_apply_deltas
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int] + \
        [ctypes.c_float] * 5 + [ctypes.c_void_p]
    w = [float(F32(x)) for x in weights]
    fn(_p(deltas), _p(boxes), N, K, *w, float(F32(scale_clamp)), _p(out))
    return out


# ------------------------------------------------------------------- glue
def area(boxes):
    """box_list_ops.area (lib/structures/box_list_ops.py:31-43)."""
    b = _f32(boxes)
    return (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])


def clip_to_window(boxes, window):
    """box_list_ops.clip_to_window, filter_nonoverlapping=False (:112-147)."""
    b = _f32(boxes)
    wy0, wx0, wy1, wx1 = [F32(v) for v in window]
    out = np.empty_like(b)
    out[:, 0] = np.maximum(np.minimum(b[:, 0], wy1), wy0)
    out[:, 1] = np.maximum(np.minimum(b[:, 1], wx1), wx0)
    out[:, 2] = np.maximum(np.minimum(b[:, 2], wy1), wy0)
    out[:, 3] = np.maximum(np.minimum(b[:, 3], wx1), wx0)
    return out


def assign_boxes_to_levels(boxes, min_level, max_level, canonical_box_size, canonical_level):
    """lib/modeling/poolers.py:11-49 (float32; log rounded from float64, so
    boxes within ~1 ulp of a level boundary may differ from any other libm)."""
    box_sizes = np.sqrt(area(boxes))
    t = box_sizes / F32(canonical_box_size) + EPS
    with np.errstate(divide="ignore", invalid="ignore"):
        lg = np.log(t.astype(np.float64)).astype(F32)
        v = F32(canonical_level) + lg / LN2
        fl = np.floor(v)
    lv = np.where(np.isfinite(fl), fl, min_level).astype(np.int64)
    lv = np.clip(lv, min_level, max_level)
    return lv - min_level


def roi_pooler(features, boxes, box_img, output_size, scales, sampling_ratio, aligned=True,
               canonical_box_size=224, canonical_level=4):
    """ROIPooler.call (lib/modeling/poolers.py:134-180): per level where/gather,
    ROIAlign, concat, invert_permutation."""
    boxes, box_img = _f32(boxes).reshape(-1, 4), _i32(box_img)
    if len(features) == 1:
        return roi_align(features[0], boxes, box_img, output_size, scales[0], sampling_ratio,
                         aligned), np.zeros(boxes.shape[0], np.int64)
    min_level = int(round(-math.log2(scales[0])))
    max_level = int(round(-math.log2(scales[-1])))
    lv = assign_boxes_to_levels(boxes, min_level, max_level, canonical_box_size, canonical_level)
    C = features[0].shape[-1]
    out = np.zeros((boxes.shape[0], output_size[0], output_size[1], C), F32)
    for level, (x, s) in enumerate(zip(features, scales)):
        inds = np.where(lv == level)[0]
        if inds.size == 0:
            continue
        out[inds] = roi_align(x, boxes[inds], box_img[inds], output_size, s, sampling_ratio,
                              aligned)
    return out, lv


def generate_cell_anchors(sizes, aspect_ratios):
    """DefaultAnchorGenerator.generate_cell_anchors (anchor_generator.py:111-144):
    python float64 arithmetic, then tf.convert_to_tensor(float32)."""
    anchors = []
    for size in sizes:
        area_ = size ** 2.0
        for aspect_ratio in aspect_ratios:
            w = math.sqrt(area_ / aspect_ratio)
            h = aspect_ratio * w
            anchors.append([-h / 2.0, -w / 2.0, h / 2.0, w / 2.0])
    return np.array(anchors, dtype=F32)


def grid_anchors(H, W, stride, cell):
    """anchor_generator.py:31-40 + :92-109; order [H, W, A]."""
    sy = (np.arange(H, dtype=np.int64) * stride).astype(F32)
    sx = (np.arange(W, dtype=np.int64) * stride).astype(F32)
    shift_x, shift_y = np.meshgrid(sx, sy)
    shift_y, shift_x = shift_y.reshape(-1), shift_x.reshape(-1)
    shifts = np.stack([shift_y, shift_x, shift_y, shift_x], axis=1)
    return (shifts[:, None, :] + cell[None, :, :].astype(F32)).reshape(-1, 4).astype(F32)


def softmax(x):
    """tf.nn.softmax on CPU: exp(x - max) * (1 / sum)."""
    x = _f32(x)
    e = np.exp(x - x.max(axis=-1, keepdims=True))
    return e * (F32(1.0) / e.sum(axis=-1, keepdims=True, dtype=F32))


def sigmoid(x):
    x = _f32(x)
    return (F32(1.0) / (F32(1.0) + np.exp(-x))).astype(F32)


def find_top_rpn_proposals(proposals, logits, image_shapes, nms_thresh, pre_nms_topk,
                           post_nms_topk, min_box_side_len):
    """rpn_outputs.py:29-132.  proposals[l] [N, HWA, 4], logits[l] [N, HWA],
    image_shapes [N, 2].  Returns boxes [N, post, 4], scores [N, post], valid."""
    N = logits[0].shape[0]
    ob = np.zeros((N, post_nms_topk, 4), F32)
    os_ = np.zeros((N, post_nms_topk), F32)
    ov = np.zeros((N, post_nms_topk), bool)
    for n in range(N):
        pb, ps = [], []
        for props_l, logit_l in zip(proposals, logits):
            k = min(pre_nms_topk, logit_l.shape[1])
            sc, idx = top_k(logit_l[n], k)
            bx = props_l[n][idx]
            h, w = image_shapes[n]
            bx = clip_to_window(bx, [0, 0, h, w])
            if min_box_side_len > 0:
                hh, ww = bx[:, 2] - bx[:, 0], bx[:, 3] - bx[:, 1]
                ok = np.where((ww >= F32(min_box_side_len)) & (hh >= F32(min_box_side_len)))[0]
                bx, sc = bx[ok], sc[ok]
            keep = nms(bx, sc, post_nms_topk, nms_thresh)
            pb.append(bx[keep])
            ps.append(sc[keep])
        pb, ps = np.concatenate(pb, 0), np.concatenate(ps, 0)
        k = min(ps.shape[0], post_nms_topk)
        sc, idx = top_k(ps, k)
        ob[n, :k] = pb[idx]
        os_[n, :k] = sc
        ov[n, :k] = True
    return ob, os_, ov


def fast_rcnn_inference(boxes, probs, roi_img, roi_slot, P, image_shapes, score_thresh,
                        nms_thresh, topk_per_image, nms_cls_agnostic=False):
    """fast_rcnn.py:28-187 (class-specific boxes; nms_cls_agnostic: plain NMS
    over the filtered boxes, fast_rcnn.py:138-139).  boxes [R, K*4] decoded,
    probs [R, K+1], (roi_img, roi_slot) the SparseBoxList indices, P dense
    slots per image.  Returns per image (boxes, scores, classes, valid, roi)."""
    boxes, probs = _f32(boxes), _f32(probs)
    R = probs.shape[0]
    K = probs.shape[1] - 1
    N = len(image_shapes)
    scores = probs[:, :-1]
    dense_b = np.zeros((N, P, K, 4), F32)
    dense_s = np.zeros((N, P, K), F32)
    dense_b[roi_img, roi_slot] = boxes.reshape(R, K, 4)
    dense_s[roi_img, roi_slot] = scores
    slot2roi = -np.ones((N, P), np.int64)
    slot2roi[roi_img, roi_slot] = np.arange(R)
    res = []
    for n in range(N):
        h, w = image_shapes[n]
        bx = clip_to_window(dense_b[n].reshape(-1, 4), [0, 0, h, w]).reshape(P, K, 4)
        bx = bx.transpose(1, 0, 2)           # [K, P, 4]
        sc = dense_s[n].transpose(1, 0)      # [K, P]
        filt = np.argwhere(sc > F32(score_thresh))   # class-major tf.where order
        fb = bx[filt[:, 0], filt[:, 1]]
        fs = sc[filt[:, 0], filt[:, 1]]
        max_coord = bx.max() if bx.size else F32(0)
        offsets = filt[:, 0].astype(F32)[:, None] * (max_coord + F32(1))
        keep = nms(fb if nms_cls_agnostic else fb + offsets, fs, topk_per_image, nms_thresh)
        ob = np.zeros((topk_per_image, 4), F32)
        osc = np.zeros(topk_per_image, F32)
        oc = np.zeros(topk_per_image, np.int64)
        ov = np.zeros(topk_per_image, bool)
        oroi = -np.ones(topk_per_image, np.int64)
        m = len(keep)
        ob[:m], osc[:m], oc[:m], ov[:m] = fb[keep], fs[keep], filt[keep, 0], True
        oroi[:m] = slot2roi[n, filt[keep, 1]]
        res.append((ob, osc, oc, ov, oroi))
    return res


def retinanet_inference(box_cls, box_delta, anchors, num_classes, topk_candidates,
                        score_threshold, nms_threshold, max_detections, weights,
                        scale_clamp=DEFAULT_SCALE_CLAMP):
    """RetinaNetHead.inference (retinanet.py:285-387).  box_cls[l] [N, HWA, K]
    logits, box_delta[l] [N, HWA, 4], anchors[l] [HWA, 4]."""
    N = box_cls[0].shape[0]
    out = []
    for n in range(N):
        ba, sa, ca = [], [], []
        for cls_l, d_l, a_l in zip(box_cls, box_delta, anchors):
            p = sigmoid(cls_l[n].reshape(-1))
            k = min(topk_candidates, d_l.shape[1])
            prob, idx = top_k(p, k)
            keep = np.where(prob > F32(score_threshold))[0]
            prob, idx = prob[keep], idx[keep]
            aidx, cidx = idx // num_classes, idx % num_classes
            boxes = apply_deltas(d_l[n][aidx], a_l[aidx], weights, scale_clamp)
            ba.append(boxes)
            sa.append(prob)
            ca.append(cidx)
        ba, sa, ca = np.concatenate(ba), np.concatenate(sa), np.concatenate(ca)
        max_coord = ba.max() if ba.size else F32(-np.inf)
        offs = ca.astype(F32) * (max_coord + F32(1))
        keep = nms(ba + offs[:, None], sa, max_detections, nms_threshold)
        ob = np.zeros((max_detections, 4), F32)
        osc = np.zeros(max_detections, F32)
        oc = np.zeros(max_detections, np.int32)
        ov = np.zeros(max_detections, bool)
        m = len(keep)
        ob[:m], osc[:m], oc[:m], ov[:m] = ba[keep], sa[keep], ca[keep], True
        out.append((ob, osc, oc, ov))
    return out


def matrix_nms(masks, classes, scores, sum_masks=None, kernel="gaussian", sigma=2.0):
    """lib/layers/nms.py:29-83, float32 numpy (matmul in float64 then rounded:
    exact for 0/1 masks)."""
    masks = _f32(masks)
    n = masks.shape[0]
    if sum_masks is None:
        sum_masks = masks.reshape(n, -1).sum(axis=1, dtype=np.float64).astype(F32)
    m = masks.reshape(n, -1).astype(np.float64)
    inter = (m @ m.T).astype(F32)
    sum_matrix = np.tile(sum_masks[None, :], (n, 1)).astype(F32)
    union = sum_matrix + sum_matrix.T - inter
    with np.errstate(divide="ignore", invalid="ignore"):
        iou = inter / union
    iou = iou - np.tril(iou)
    cls = np.asarray(classes)
    cmat = (cls[None, :] == cls[:, None]).astype(F32)
    iou = iou * cmat
    # reduce_max / reduce_min: Eigen's scalar Max/MinReducer update only when
    # `t < accum` (`t > accum`) holds, i.e. they skip NaN (the linear kernel's
    # 0 / 0 where comp = 1 and iou = 1): fmax / fmin reductions
    comp = np.fmax.reduce(iou, axis=0)
    comp = np.tile(comp[None, :], (n, 1)).T
    if kernel == "gaussian":
        decay = np.exp(F32(-1 * sigma) * (iou ** 2 - comp ** 2))
    elif kernel == "linear":
        decay = (F32(1.0) - iou) / (F32(1.0) - comp)
    else:
        raise NotImplementedError(kernel)
    return (_f32(scores) * np.fmin.reduce(decay, axis=0)).astype(F32)


def paste_masks(box_masks, boxes, out_shape, valid=None, yx_scale=None, threshold=0.5):
    """detector_postprocess -> reframe_box_masks_to_image_masks
    (lib/modeling/postprocessing.py:33-50, lib/structures/mask_ops.py:7-56),
    float32 numpy glue around the C CropAndResize:
      box_list_ops.scale (fixed format, :86-108) -> to_normalized_coordinates
      (:806-839, scale by 1/H, 1/W) -> reverse box of the unit square
      (mask_ops.py:37-49) -> tf.image.crop_and_resize(crop = canvas) -> tf.greater.
    box_masks [D, mh, mw], boxes [D, 4] yxyx absolute; returns [D, H, W] uint8
    (rows with valid False are zeros, SparseBoxList.to_dense)."""
    m = _f32(box_masks)
    b = _f32(boxes).reshape(-1, 4).copy()
    D = b.shape[0]
    H, W = int(out_shape[0]), int(out_shape[1])
    if yx_scale is not None:
        s = _f32(yx_scale).reshape(-1, 2)
        b[:, 0] = s[:, 0] * b[:, 0]
        b[:, 2] = s[:, 0] * b[:, 2]
        b[:, 1] = s[:, 1] * b[:, 1]
        b[:, 3] = s[:, 1] * b[:, 3]
    ih, iw = F32(1) / F32(H), F32(1) / F32(W)
    b[:, 0] = ih * b[:, 0]
    b[:, 2] = ih * b[:, 2]
    b[:, 1] = iw * b[:, 1]
    b[:, 3] = iw * b[:, 3]
    lo, hi = b[:, 0:2], b[:, 2:4]
    unit = np.array([[0, 0], [1, 1]], F32)
    rev = ((unit[None] - lo[:, None, :]) / (hi - lo)[:, None, :]).reshape(-1, 4).astype(F32)
    out = np.zeros((D, H, W), np.uint8)
    keep = np.arange(D) if valid is None else np.flatnonzero(np.asarray(valid))
    if keep.size:
        crops = crop_and_resize_tf(m[keep][..., None], rev[keep], np.arange(keep.size), (H, W))
        out[keep] = (crops[..., 0] > F32(threshold)).astype(np.uint8)
    return out
