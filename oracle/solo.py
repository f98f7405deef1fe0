"""ORACLE — test infrastructure only (never imported by the product path).

float32 numpy restatement of the SOLOv2 inference tail
(lib/modeling/single_stage_heads/solo_v2.py) and of the TF ResizeBilinear
kernel the head resamples with (lib/layers/functional.py:9-36: TF >= 1.14
takes the tf.compat.v2.image.resize branch, whose kwargs filter drops
align_corners — half-pixel centres, no antialias; TF 1.15
resize_bilinear_op.cc arithmetic).  Each function cites the reference lines
it follows.  The top-k and Matrix NMS are the oracle's (oracle.py:
TopKV2 order, nms.py:29-83).

Parity status: pinned by hand-computed known answers only (tests/test_oracle.py
and tests/test_solo.py: bilinear sample weights, linspace, point NMS, the
box-from-mask rule); the reference ships no SOLO fixtures and TensorFlow
cannot run here — "parity unpinned" against TensorFlow itself.
"""
import numpy as np

import oracle

F32 = np.float32


def linspace_tf(num):
    """tf.linspace(-1., 1., num), float32 (LinSpaceOp: start + step * i, last = stop)."""
    if num == 1:
        return np.array([-1.0], F32)
    step = F32(2.0) / F32(num - 1)
    a = F32(-1.0) + step * np.arange(num, dtype=F32)
    a[-1] = F32(1.0)
    return a.astype(F32)


def coord_channels(N, H, W):
    """(xx, yy) channels of solo_v2.py:258-262 / :712-716: [N, H, W, 2]."""
    xx, yy = np.meshgrid(linspace_tf(W), linspace_tf(H))
    c = np.stack([xx, yy], axis=-1).astype(F32)
    return np.broadcast_to(c[None], (N, H, W, 2)).copy()


def _interp(out_size, in_size, half_pixel=True, align_corners=False):
    """compute_interpolation_weights (resize_bilinear_op.cc): lower, upper, lerp."""
    if align_corners and out_size > 1:
        scale = F32(in_size - 1) / F32(out_size - 1)
    else:
        scale = F32(in_size) / F32(out_size)
    i = np.arange(out_size, dtype=F32)
    if half_pixel:
        v = (i + F32(0.5)) * scale - F32(0.5)
    else:
        v = i * scale
    v = v.astype(F32)
    f = np.floor(v)
    lo = np.maximum(f.astype(np.int64), 0)
    hi = np.minimum(np.ceil(v).astype(np.int64), in_size - 1)
    return lo, hi, (v - f).astype(F32)


def resize_bilinear_tf(x, oh, ow, half_pixel=True, align_corners=False):
    """TF ResizeBilinear, NHWC float32: compute_lerp
    top = tl + (tr - tl) * xl, bottom = bl + (br - bl) * xl,
    out = top + (bottom - top) * yl."""
    x = np.asarray(x, F32)
    N, H, W, C = x.shape
    ylo, yhi, yl = _interp(oh, H, half_pixel, align_corners)
    xlo, xhi, xl = _interp(ow, W, half_pixel, align_corners)
    top_rows, bot_rows = x[:, ylo], x[:, yhi]             # [N, oh, W, C]
    tl, tr = top_rows[:, :, xlo], top_rows[:, :, xhi]    # [N, oh, ow, C]
    bl, br = bot_rows[:, :, xlo], bot_rows[:, :, xhi]
    xl_ = xl[None, None, :, None]
    yl_ = yl[None, :, None, None]
    top = tl + (tr - tl) * xl_
    bottom = bl + (br - bl) * xl_
    return (top + (bottom - top) * yl_).astype(F32)


def point_nms(p):
    """point_nms (solo_v2.py:29-40) on sigmoid maps [N, S, S, K]: zero pad 1,
    2x2 stride-1 VALID max pool, keep where p equals the window max."""
    p = np.asarray(p, F32)
    pad = np.pad(p, ((0, 0), (1, 1), (1, 1), (0, 0)))
    m = np.maximum(np.maximum(pad[:, :-1, :-1], pad[:, :-1, 1:]),
                   np.maximum(pad[:, 1:, :-1], pad[:, 1:, 1:]))
    keep = (p == m[:, :-1, :-1]).astype(F32)
    return (p * keep).astype(F32)


def cell_strides(grids, strides):
    """The per-cell stride vector of solo_v2.py:490-497."""
    return np.concatenate([np.full(g * g, s, F32) for g, s in zip(grids, strides)])


def inference_single_image(probs, cell_logits, strides, score_thr=0.1, mask_thr=0.5,
                           update_thr=0.05, pre_nms_topk=500, max_det=100, kernel="gaussian",
                           sigma=2.0):
    """inference_single_image (solo_v2.py:478-565).  probs [T, K] (sigmoid +
    point NMS, flattened over levels), cell_logits(cells) -> [n, P] mask logits
    of the dynamic 1x1 conv for those cells (:499-511), strides [T].
    Returns masks [max_det, P] f32 0/1, classes int64, scores, is_valid, and
    a dict of intermediates."""
    probs = np.asarray(probs, F32)
    keep = np.argwhere(probs > F32(score_thr))          # tf.where: (cell, class) row-major
    scores = probs[keep[:, 0], keep[:, 1]]
    labels = keep[:, 1].astype(np.int64)
    cells = keep[:, 0]
    st = np.asarray(strides, F32)[cells]
    logits = np.asarray(cell_logits(cells), F32)
    sig = oracle.sigmoid(logits)
    masks = (sig > F32(mask_thr)).astype(F32)
    sum_masks = masks.sum(axis=1, dtype=np.float64).astype(F32)   # exact (0/1 counts)
    kb = sum_masks > st
    masks, sig, scores, labels, sum_masks, cells = (masks[kb], sig[kb], scores[kb], labels[kb],
                                                    sum_masks[kb], cells[kb])
    mask_scoring = ((sig * masks).sum(axis=1, dtype=F32) / sum_masks).astype(F32)
    scores = (scores * mask_scoring).astype(F32)
    k = min(pre_nms_topk, scores.shape[0])
    sc, idx = oracle.top_k(scores, k)
    masks, sum_masks, labels, cells = masks[idx], sum_masks[idx], labels[idx], cells[idx]
    dec = oracle.matrix_nms(masks, labels, sc, sum_masks, kernel, sigma) if k else sc
    kb = dec > F32(update_thr)
    P = masks.shape[1] if masks.ndim == 2 else 0
    out_m = np.zeros((max_det, P), F32)
    out_c = np.zeros(max_det, np.int64)
    out_s = np.zeros(max_det, F32)
    out_v = np.zeros(max_det, bool)
    m = min(int(kb.sum()), max_det)
    out_m[:m], out_c[:m], out_s[:m], out_v[:m] = masks[kb][:m], labels[kb][:m], dec[kb][:m], True
    info = {"num_candidates": int(keep.shape[0]), "top_scores": sc, "top_classes": labels,
            "top_cells": cells, "top_sum_masks": sum_masks, "decayed": dec}
    return out_m, out_c, out_s, out_v, info


def masks_to_image(masks, Hm, Wm, OH, OW, mask_thr=0.5):
    """solo_v2.py:598-623 for one image: masks [D, Hm*Wm] 0/1 -> resize to
    [OH, OW] (TF bilinear, half-pixel), > thr; boxes: yy = mask * y, the zeros
    replaced by sum(yy) / (sum(mask) + 1e-5), then min / max (sums in float64,
    rounded once to float32: the GPU's exact integer sums)."""
    D = masks.shape[0]
    m = np.asarray(masks, F32).reshape(D, Hm, Wm).transpose(1, 2, 0)[None]
    r = resize_bilinear_tf(m, OH, OW)[0].transpose(2, 0, 1)    # [D, OH, OW]
    on = r > F32(mask_thr)
    boxes = np.zeros((D, 4), F32)
    ys = np.arange(OH, dtype=np.float64)
    xs = np.arange(OW, dtype=np.float64)
    for d in range(D):
        md = on[d]
        cnt = F32(md.sum())
        sy = F32((md.sum(axis=1) * ys).sum())
        sx = F32((md.sum(axis=0) * xs).sum())
        den = F32(cnt + F32(1e-5))
        ym, xm = F32(sy / den), F32(sx / den)
        rows = np.nonzero(md.any(axis=1))[0]
        cols = np.nonzero(md.any(axis=0))[0]
        rows, cols = rows[rows > 0], cols[cols > 0]
        ymin = min(ym, F32(rows.min())) if rows.size else ym
        ymax = max(ym, F32(rows.max())) if rows.size else ym
        xmin = min(xm, F32(cols.min())) if cols.size else xm
        xmax = max(xm, F32(cols.max())) if cols.size else xm
        boxes[d] = (ymin, xmin, ymax, xmax)
    return on.astype(np.uint8), boxes
