"""ORACLE (training targets and losses) — test infrastructure only.

Per-image numpy restatement of the reference's training-target glue, written
the way the reference writes it (boolean_mask of the valid GT, one image at a
time, dynamic_stitch of label groups), so the batched/dense GPU versions in
detectron2_tensorflow_amd.modeling can be checked against it.  float32
throughout.  Randomness (subsample_labels' random_shuffle) is not restated:
tests use inputs where every candidate is sampled, which makes the reference
deterministic.

Parity status: restated from the reference source (cited per function);
unpinned by reference-run vectors (TensorFlow cannot run here).
"""
import numpy as np

from oracle import crop_and_resize_tf

F32 = np.float32


def pairwise_iou(b1, b2):
    """box_list_ops.py:295-331 (iou_type 'iou')."""
    b1 = np.asarray(b1, F32).reshape(-1, 4)
    b2 = np.asarray(b2, F32).reshape(-1, 4)
    ih = np.maximum(F32(0), np.minimum(b1[:, None, 2], b2[None, :, 2]) -
                    np.maximum(b1[:, None, 0], b2[None, :, 0]))
    iw = np.maximum(F32(0), np.minimum(b1[:, None, 3], b2[None, :, 3]) -
                    np.maximum(b1[:, None, 1], b2[None, :, 1]))
    inter = ih * iw
    a1 = (b1[:, 2] - b1[:, 0]) * (b1[:, 3] - b1[:, 1])
    a2 = (b2[:, 2] - b2[:, 0]) * (b2[:, 3] - b2[:, 1])
    union = a1[:, None] + a2[None, :] - inter
    with np.errstate(divide="ignore", invalid="ignore"):
        iou = np.where(union == 0, F32(0), inter / union).astype(F32)
    return iou


def matcher(quality, thresholds, labels, allow_low_quality_matches, crowd=None, difficult=None):
    """Matcher.__call__ (matcher.py:55-139) on an [M, N] matrix of VALID GT."""
    thr = [-np.inf] + list(thresholds) + [np.inf]
    M, N = quality.shape
    if M > 0:
        matches = np.argmax(quality, axis=0).astype(np.int64)
        vals = quality.max(axis=0)
        lab = np.zeros(N, np.int64)
        for lb, lo, hi in zip(labels, thr[:-1], thr[1:]):
            lab[(vals >= lo) & (vals < hi)] = lb
        if allow_low_quality_matches:
            # get_low_quality_matches_ (matcher.py:141-173), ties included
            best = quality.max(axis=1)
            _, preds = np.nonzero(quality == best[:, None])
            lab[preds] = 1
    else:
        matches = np.zeros(N, np.int64)
        lab = np.zeros(N, np.int64)
    if crowd is not None and crowd.shape[0] > 0:
        lab[(lab == 0) & (crowd.max(axis=0) > 1e-3)] = -1
    if difficult is not None and difficult.shape[0] > 0:
        lab[(lab == 0) & (difficult.max(axis=0) > thr[1])] = -1
    return matches, lab


def get_deltas(src, tgt, weights):
    """Box2BoxTransform.get_deltas (box_regression.py:38-74)."""
    src = np.asarray(src, F32)
    tgt = np.asarray(tgt, F32)
    sh = src[:, 2] - src[:, 0]
    sw = src[:, 3] - src[:, 1]
    scy = src[:, 0] + F32(0.5) * sh
    scx = src[:, 1] + F32(0.5) * sw
    th = tgt[:, 2] - tgt[:, 0]
    tw = tgt[:, 3] - tgt[:, 1]
    tcy = tgt[:, 0] + F32(0.5) * th
    tcx = tgt[:, 1] + F32(0.5) * tw
    wy, wx, wh, ww = [F32(w) for w in weights]
    return np.stack([wy * (tcy - scy) / sh, wx * (tcx - scx) / sw,
                     wh * np.log(th / sh), ww * np.log(tw / sw)], 1).astype(F32)


def rpn_targets(anchors, gt_boxes, is_valid, is_crowd, weights, thresholds, labels,
                image_shape=None, boundary_threshold=-1):
    """RPNOutputs._get_ground_truth, one image (rpn_outputs.py:255-290)."""
    valid = is_valid & ~is_crowd
    vgt = gt_boxes[valid]
    iou = pairwise_iou(vgt, anchors)
    crowd = pairwise_iou(gt_boxes[is_crowd], anchors)
    matches, lab = matcher(iou, thresholds, labels, True, crowd)
    if boundary_threshold >= 0:
        t = boundary_threshold
        inside = ~((anchors[:, 0] < -t) | (anchors[:, 1] < -t) |
                   (anchors[:, 2] > image_shape[0] + t) | (anchors[:, 3] > image_shape[1] + t))
        lab = np.where(inside, lab, -1)
    deltas = np.zeros_like(anchors, dtype=F32)
    pos = np.nonzero(lab > 0)[0]
    if len(pos):
        deltas[pos] = get_deltas(anchors[pos], vgt[matches[pos]], weights)
    return lab, deltas


def rpn_losses(labels, gt_deltas, pred_logits, pred_deltas, num_images, batch_size_per_image):
    """rpn_losses (rpn_outputs.py:135-185) with beta = 0 plus the normaliser
    (:396-399); labels already subsampled (-1 = not sampled)."""
    pos = labels == 1
    loc = np.abs(gt_deltas[pos] - pred_deltas[pos]).astype(np.float64).sum()
    v = labels >= 0
    x = pred_logits[v].astype(np.float64)
    z = labels[v].astype(np.float64)
    # sigmoid_cross_entropy_with_logits: max(x, 0) - x * z + log(1 + exp(-|x|))
    obj = (np.maximum(x, 0) - x * z + np.log1p(np.exp(-np.abs(x)))).sum()
    norm = 1.0 / (batch_size_per_image * num_images)
    return obj * norm, loc * norm


def retinanet_targets(anchors, gt_boxes, gt_classes, is_valid, num_classes, weights,
                      thresholds=(0.4, 0.5), labels=(0, -1, 1)):
    """RetinaNet.get_ground_truth, one image (retinanet.py:212-283): the
    valid GT (boolean_mask) against every anchor, Matcher with low-quality
    matches; classes = matched GT class (label 1), K (label 0), -1 (ignored);
    deltas = get_deltas(anchor, matched GT) for the positives, else 0."""
    valid = np.asarray(is_valid, bool)
    vgt = np.asarray(gt_boxes, F32)[valid]
    vcls = np.asarray(gt_classes, np.int64)[valid]
    iou = pairwise_iou(vgt, anchors)
    matches, lab = matcher(iou, thresholds, labels, True)
    cls = np.full(len(anchors), -1, np.int64)
    pos = np.nonzero(lab > 0)[0]
    cls[lab == 0] = num_classes
    cls[pos] = vcls[matches[pos]]
    deltas = np.zeros((len(anchors), 4), F32)
    if len(pos):
        deltas[pos] = get_deltas(anchors[pos], vgt[matches[pos]], weights)
    return cls, deltas


def sigmoid_focal_loss(x, t, alpha, gamma):
    """loss.py:59-101 elementwise, float64."""
    x = np.asarray(x, np.float64)
    t = np.asarray(t, np.float64)
    p = 1.0 / (1.0 + np.exp(-x))
    ce = np.maximum(x, 0) - x * t + np.log1p(np.exp(-np.abs(x)))
    p_t = p * t + (1 - p) * (1 - t)
    loss = ce * (1 - p_t) ** gamma
    if alpha >= 0:
        loss = (alpha * t + (1 - alpha) * (1 - t)) * loss
    return loss


def retinanet_losses(gt_classes, gt_deltas, logits, deltas, num_classes, alpha, gamma, beta,
                     normalizer, momentum=0.9):
    """RetinaNet.losses (retinanet.py:147-210) over the batch's [N*R] anchor
    rows: focal "sum" over the valid rows' one-hot targets, smooth-L1 "sum"
    over the foreground rows, both / the normaliser EMA after its update
    (assign_moving_average, zero_debias=False).  Returns (cls, box, new
    normaliser), float64."""
    gt_classes = np.asarray(gt_classes).reshape(-1)
    logits = np.asarray(logits).reshape(-1, num_classes)
    deltas = np.asarray(deltas).reshape(-1, 4)
    gt_deltas = np.asarray(gt_deltas).reshape(-1, 4)
    valid = gt_classes >= 0
    fg = valid & (gt_classes < num_classes)
    onehot = np.zeros_like(logits, dtype=np.float64)
    onehot[np.nonzero(fg)[0], gt_classes[fg]] = 1.0
    cls = sigmoid_focal_loss(logits[valid], onehot[valid], alpha, gamma).sum()
    n = np.abs(gt_deltas[fg].astype(np.float64) - deltas[fg].astype(np.float64))
    l1 = n if beta < 1e-5 else np.where(n < beta, 0.5 * n ** 2 / beta, n - 0.5 * beta)
    nfg = max(1.0, float(fg.sum()))
    norm = normalizer - (normalizer - nfg) * (1 - momentum)
    return cls / norm, l1.sum() / norm, norm


def label_proposals(proposals, p_valid, gt_boxes, gt_classes, is_valid, is_crowd, difficult,
                    num_classes, iou_threshold, append_gt=True):
    """label_and_sample_proposals before sampling, one image (roi_heads.py:130-180).
    Returns (kept proposal boxes, gt_classes per proposal, matched GT box)."""
    if append_gt:  # proposal_utils.py:31-45 (all GT rows appended, validity kept)
        proposals = np.concatenate([proposals, gt_boxes])
        p_valid = np.concatenate([p_valid, is_valid])
    vb = is_valid & ~is_crowd & ~difficult
    vgt, vcls = gt_boxes[vb], gt_classes[vb]
    props = proposals[p_valid]
    iou = pairwise_iou(vgt, props)
    matches, lab = matcher(iou, [iou_threshold], [0, 1], False,
                           pairwise_iou(gt_boxes[is_crowd], props),
                           pairwise_iou(gt_boxes[difficult], props))
    cls = np.full(len(props), -1, np.int64)
    cls[lab == 1] = vcls[matches[lab == 1]] if len(vcls) else 0
    cls[lab == 0] = num_classes
    mgt = vgt[matches] if len(vgt) else np.zeros_like(props)
    return props, cls, mgt


def fast_rcnn_losses(logits, deltas, proposals, gt_classes, gt_boxes, weights):
    """FastRCNNOutputs.losses (fast_rcnn.py:269-357), beta = 0, over the valid rows."""
    R = len(gt_classes)
    if R == 0:
        return 0.0, 0.0
    x = logits.astype(np.float64)
    m = x.max(axis=1, keepdims=True)
    lse = (m[:, 0] + np.log(np.exp(x - m).sum(axis=1)))
    loss_cls = (lse - x[np.arange(R), gt_classes]).mean()
    K = logits.shape[1] - 1
    fg = (gt_classes >= 0) & (gt_classes < K)
    if not fg.any():
        return loss_cls, 0.0
    nreg = deltas.shape[1] // 4
    d = deltas.reshape(R, nreg, 4)
    col = gt_classes[fg] if nreg > 1 else np.zeros(fg.sum(), np.int64)
    pred = d[np.nonzero(fg)[0], col]
    tgt = get_deltas(proposals[fg], gt_boxes[fg], weights)
    return loss_cls, np.abs(tgt - pred).astype(np.float64).sum() / R


def mask_rcnn_loss(logits, boxes, gt_boxes, gt_classes, gt_masks):
    """mask_rcnn_loss (mask_head.py:17-68) with mini masks: logits [B, Hm, Wm, C],
    boxes / gt_boxes [B, 4], gt_masks [B, h, w] (the matched mini mask per row)."""
    B, Hm, Wm, C = logits.shape
    if B == 0:
        return 0.0
    y1, x1, y2, x2 = [boxes[:, i] for i in range(4)]
    gy1, gx1, gy2, gx2 = [gt_boxes[:, i] for i in range(4)]
    gh, gw = gt_boxes[:, 2] - gy1, gt_boxes[:, 3] - gx1
    nb = np.stack([(y1 - gy1) / gh, (x1 - gx1) / gw, (y2 - gy1) / gh, (x2 - gx1) / gw],
                  1).astype(F32)
    tgt = crop_and_resize_tf(gt_masks.astype(F32)[..., None], nb, np.arange(B, dtype=np.int32),
                             (Hm, Wm))[..., 0]
    tgt = np.round(tgt).astype(np.float64)
    ch = gt_classes if C > 1 else np.zeros(B, np.int64)
    x = logits[np.arange(B), :, :, ch].astype(np.float64)
    return (np.maximum(x, 0) - x * tgt + np.log1p(np.exp(-np.abs(x)))).mean()


def sgd_step(params, grads, accums, lr, momentum, weight_decays, clip_norm):
    """One reference update: grad of loss + sum(wd * |w|^2 / 2), per-tensor
    clip_by_norm (slim.learning.clip_gradient_norms), MomentumOptimizer."""
    out_p, out_a = [], []
    for p, g, a, wd in zip(params, grads, accums, weight_decays):
        g = g.astype(np.float64) + wd * p.astype(np.float64)
        n = np.sqrt((g * g).sum())
        if clip_norm > 0:
            g = g * clip_norm / max(n, clip_norm)
        a = momentum * a + g
        out_a.append(a)
        out_p.append(p - lr * a)
    return out_p, out_a


def _floordiv_f32(x, g):
    """TF FloorDiv of a float32 tensor by the Python float 1. / g (converted
    to float32): floor(x / f32(1 / g)) in float32 (solo_v2.py:402-435)."""
    q = (np.asarray(x, F32) / F32(1.0 / g)).astype(F32)
    return np.floor(q).astype(F32)


def solov2_targets(gt_boxes, gt_classes, is_valid, gt_masks, mask_hw, num_grids, scale_ranges,
                   sigma):
    """MaskKernelBranch.get_ground_truth (solo_v2.py:373-474) for a dense
    batch: gt_boxes [N, G, 4] yxyx image px, gt_classes [N, G], is_valid
    [N, G], gt_masks [N, G, Hi, Wi] 0/1 at the padded image size, mask_hw the
    mask-feature size.  The valid GT in batch-major order (SparseBoxList.from_dense).
    Per level: (grid classes [N, S, S] int64 with 0 = no object, positive
    (batch, cell) pairs [P, 2] in tf.where order -- GT, then row, then column --
    and their target masks [P, Hm, Wm] float32).

    center_of_mass is the reference's (:43-64): the MEAN of mask * coordinate
    over every pixel (not divided by the mask area), here from exact sums
    (float64) rounded to float32 -- TF's float32 reduce_mean over ~1 M pixels
    depends on its summation order.  A cell claimed by two GT of one level
    takes the later GT's class (tf.sparse.reorder + to_dense keep one of the
    duplicates; which one is unpinned)."""
    gt_boxes = np.asarray(gt_boxes, F32)
    N, G = gt_boxes.shape[:2]
    vb, vg = np.nonzero(np.asarray(is_valid, bool))
    boxes = gt_boxes[vb, vg]
    classes = np.asarray(gt_classes)[vb, vg].astype(np.int64)
    masks = np.asarray(gt_masks)[vb, vg].astype(F32)
    h = (boxes[:, 2] - boxes[:, 0]).astype(F32)
    w = (boxes[:, 3] - boxes[:, 1]).astype(F32)
    area_sqrt = np.sqrt((h * w).astype(F32)).astype(F32)
    half_h = (F32(0.5) * h * F32(sigma)).astype(F32)
    half_w = (F32(0.5) * w * F32(sigma)).astype(F32)
    Hm, Wm = mask_hw
    up_h, up_w = F32(Hm * 4), F32(Wm * 4)
    Hi, Wi = masks.shape[1:] if len(masks) else (Hm * 4, Wm * 4)
    out = []
    for (lo, hi), S in zip(scale_ranges, num_grids):
        li = np.nonzero((area_sqrt >= F32(lo)) & (area_sqrt <= F32(hi)))[0]
        cls_map = np.zeros((N, S, S), np.int64)
        pos, tmasks = [], []
        if len(li):
            m = masks[li]
            yy = np.arange(Hi, dtype=np.float64)[None, :, None]
            xx = np.arange(Wi, dtype=np.float64)[None, None, :]
            ch = ((m.astype(np.float64) * yy).sum((1, 2)) / (Hi * Wi)).astype(F32)
            cw = ((m.astype(np.float64) * xx).sum((1, 2)) / (Hi * Wi)).astype(F32)
            coord_h = _floordiv_f32(ch / up_h, S)
            coord_w = _floordiv_f32(cw / up_w, S)
            top = np.maximum(coord_h - 1, np.maximum(F32(0), _floordiv_f32((ch - half_h[li]) / up_h, S)))
            down = np.minimum(coord_h + 1, np.minimum(F32(S - 1), _floordiv_f32((ch + half_h[li]) / up_h, S)))
            left = np.maximum(coord_w - 1, np.maximum(F32(0), _floordiv_f32((cw - half_w[li]) / up_w, S)))
            right = np.minimum(coord_w + 1, np.minimum(F32(S - 1), _floordiv_f32((cw + half_w[li]) / up_w, S)))
            rs = oracle_resize_masks(m, Hm, Wm)
            for k, gi in enumerate(li):
                for y in range(S):
                    for x in range(S):
                        if top[k] <= y <= down[k] and left[k] <= x <= right[k]:
                            b = vb[gi]
                            pos.append((b, y * S + x))
                            tmasks.append(rs[k])
                            cls_map[b, y, x] = classes[gi]
        out.append((cls_map, np.asarray(pos, np.int64).reshape(-1, 2),
                    np.asarray(tmasks, F32).reshape(-1, Hm, Wm)))
    return out


def oracle_resize_masks(m, Hm, Wm):
    """resize_images(masks[..., None], pred_mask_size) then tf.round
    (solo_v2.py:466-471): TF ResizeBilinear, half-pixel centres (the
    reference's kwargs filter drops align_corners), round half to even."""
    from solo import resize_bilinear_tf
    r = resize_bilinear_tf(np.asarray(m, F32)[..., None], Hm, Wm)[..., 0]
    return np.round(r).astype(F32)


def solov2_losses(pred_classes, pred_kernels, mask_feats, targets, num_classes, alpha, gamma,
                  ins_loss_weight):
    """MaskKernelBranch.losses (solo_v2.py:274-371): the dynamic 1x1 conv of
    every positive cell's kernel over its image's mask features, dice loss
    ("mean") x INS_LOSS_WEIGHT, and the focal loss ("sum") over every cell of
    every level against one_hot(class, K + 1)[:, 1:] (class 0 = no object),
    divided by (positives + 1).  Returns (loss_ins, loss_cls), float64."""
    feats = np.asarray(mask_feats, np.float64)
    N, Hm, Wm, E = feats.shape
    pred_masks, gt_masks = [], []
    logits, onehots = [], []
    num_ins = 0
    for (cls_map, pos, tm), pc, pk in zip(targets, pred_classes, pred_kernels):
        S = cls_map.shape[1]
        pk = np.asarray(pk, np.float64).reshape(N, S * S, E)
        for (b, j), t in zip(pos, tm):
            pred_masks.append(feats[b].reshape(-1, E) @ pk[b, j])
            gt_masks.append(t.reshape(-1))
        num_ins += len(pos)
        logits.append(np.asarray(pc, np.float64).reshape(-1, num_classes))
        oh = np.zeros((N * S * S, num_classes + 1))
        oh[np.arange(N * S * S), cls_map.reshape(-1)] = 1.0
        onehots.append(oh[:, 1:])
    if pred_masks:
        p = 1.0 / (1.0 + np.exp(-np.stack(pred_masks)))
        t = np.stack(gt_masks).astype(np.float64)
        a = (p * t).sum(1)
        bb = (p * p).sum(1)
        c = (t * t).sum(1)
        loss_ins = (1.0 - 2 * a / (bb + c + 1e-5)).mean()
    else:
        loss_ins = 0.0
    cls = sigmoid_focal_loss(np.concatenate(logits), np.concatenate(onehots), alpha, gamma).sum()
    return ins_loss_weight * loss_ins, cls / (num_ins + 1)
