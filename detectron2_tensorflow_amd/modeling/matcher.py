"""Matcher (lib/modeling/matcher.py:8-173) and subsample_labels
(lib/modeling/sampling.py:6-45), batched and dense on the GPU.

Everything works on padded [N, G] ground truth with an ``is_valid`` mask and
fixed-size outputs, so the training step needs no host synchronisation:
invalid GT rows never match (their IoU row is -inf), and the random subsample
picks the k smallest of per-element uniform keys among the candidates
(equivalent in distribution to tf.random_shuffle(...)[:k]).
"""
import torch

from ..layers import ops


def pairwise_iou(boxes1, boxes2):
    """box_list_ops.pairwise_iou (:295-372) batched: [N, G, 4] x [N, P, 4] -> [N, G, P];
    0 where the union is 0."""
    y1a, x1a, y2a, x2a = boxes1.unbind(-1)
    y1b, x1b, y2b, x2b = boxes2.unbind(-1)
    ih = (torch.minimum(y2a[..., :, None], y2b[..., None, :]) -
          torch.maximum(y1a[..., :, None], y1b[..., None, :])).clamp(min=0.0)
    iw = (torch.minimum(x2a[..., :, None], x2b[..., None, :]) -
          torch.maximum(x1a[..., :, None], x1b[..., None, :])).clamp(min=0.0)
    inter = ih * iw
    area_a = (y2a - y1a) * (x2a - x1a)
    area_b = (y2b - y1b) * (x2b - x1b)
    union = area_a[..., :, None] + area_b[..., None, :] - inter
    return torch.where(union == 0, torch.zeros_like(union), inter / union)


class Matcher:
    def __init__(self, thresholds, labels, allow_low_quality_matches=False):
        thresholds = [-float("inf")] + list(thresholds) + [float("inf")]
        assert all(lo <= hi for lo, hi in zip(thresholds[:-1], thresholds[1:]))
        assert all(lb in (-1, 0, 1) for lb in labels)
        assert len(labels) == len(thresholds) - 1
        self.thresholds = thresholds
        self.labels = list(labels)
        self.allow_low_quality_matches = allow_low_quality_matches

    def __call__(self, quality, gt_valid, crowd_quality=None, difficult_quality=None):
        """quality [N, G, P] (rows of invalid GT are ignored), gt_valid [N, G];
        crowd_quality / difficult_quality [N, G, P] with zero rows for GT that are
        not crowd / difficult (matcher.py:114-139).
        Returns matches [N, P] (int64 GT index) and labels [N, P] in {-1, 0, 1}."""
        q = torch.where(gt_valid[..., None], quality, torch.full_like(quality, -float("inf")))
        vals, matches = q.max(dim=1)
        any_gt = gt_valid.any(dim=1, keepdim=True)
        labels = torch.zeros_like(matches)
        for lb, lo, hi in zip(self.labels, self.thresholds[:-1], self.thresholds[1:]):
            labels = torch.where((vals >= lo) & (vals < hi), torch.full_like(labels, lb), labels)
        if self.allow_low_quality_matches:
            best = q.max(dim=2, keepdim=True).values  # [N, G, 1]
            hit = ((q == best) & gt_valid[..., None]).any(dim=1)
            labels = torch.where(hit, torch.ones_like(labels), labels)
        # no valid GT: every prediction is background (matcher.py:119-125)
        labels = torch.where(any_gt, labels, torch.zeros_like(labels))
        matches = torch.where(any_gt, matches, torch.zeros_like(matches))
        if crowd_quality is not None:
            crowd = (crowd_quality.max(dim=1).values > 1e-3) if crowd_quality.shape[1] else None
            if crowd is not None:
                labels = torch.where((labels == 0) & crowd, torch.full_like(labels, -1), labels)
        if difficult_quality is not None and difficult_quality.shape[1]:
            diff = difficult_quality.max(dim=1).values > self.thresholds[1]
            labels = torch.where((labels == 0) & diff, torch.full_like(labels, -1), labels)
        return matches, labels


def match_boxes(matcher, gt_boxes, valid, boxes, crowd=None, difficult=None):
    """pairwise_iou(gt_boxes, boxes) + matcher(...) with crowd / difficult
    quality rows (rpn_outputs.py:306-330, roi_heads.py:160-216): the GT
    matched against are the valid ones that are neither crowd nor difficult
    (valid_gt_boxlist).  On the GPU one fused HIP pass
    (ops.match_boxes_masks: no [N, G, P] IoU matrix, no mask arithmetic);
    elsewhere the tensor formulation.  boxes [P, 4] shared or [N, P, 4]."""
    N = gt_boxes.shape[0]
    if boxes.is_cuda:
        return ops.match_boxes_masks(gt_boxes, valid, boxes, matcher.thresholds,
                                     matcher.labels, matcher.allow_low_quality_matches,
                                     crowd=crowd, difficult=difficult, crowd_thr=1e-3,
                                     difficult_thr=matcher.thresholds[1])
    matchable = valid
    if crowd is not None:
        matchable = matchable & ~crowd
    if difficult is not None:
        matchable = matchable & ~difficult
    b = boxes if boxes.dim() == 3 else boxes[None].expand(N, -1, -1)
    iou = pairwise_iou(gt_boxes, b)
    zq = torch.zeros_like(iou)
    crowd_q = torch.where(crowd[..., None], iou, zq) if crowd is not None else None
    diff_q = torch.where(difficult[..., None], iou, zq) if difficult is not None else None
    return matcher(iou, matchable, crowd_q, diff_q)


# subsample on the GPU with the fused HIP sampler (d2mi_subsample: three
# launches instead of ~25 small ones per call); False: the random-key
# top-k formulation below (tests compare the two)
FUSED_SUBSAMPLE = True


def subsample_labels(labels, num_samples, positive_fraction, bg_label, generator=None,
                     order_slots=0):
    """Dense subsample_labels over [N, P]: returns (pos_mask, neg_mask) [N, P] bool
    with min(#pos, int(num_samples * fraction)) positives and
    min(#neg, num_samples - #pos_taken) negatives chosen uniformly at random.
    order_slots = S (GPU path): also (order [N, S], valid [N, S]), the selected
    indices positives first, each kind in index order."""
    N, P = labels.shape
    num_pos = int(num_samples * positive_fraction)
    if labels.is_cuda and (FUSED_SUBSAMPLE or order_slots):
        seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, device=labels.device,
                             generator=generator)
        return ops.subsample(labels, num_samples, num_pos, bg_label, seed, order_slots)
    positive = (labels != -1) & (labels != bg_label)
    negative = labels == bg_label
    keys = torch.rand((N, P), device=labels.device, generator=generator)
    pos_sel = _smallest(keys, positive, num_pos, num_pos)
    n_pos = pos_sel.sum(dim=1, keepdim=True)
    neg_keys = torch.rand((N, P), device=labels.device, generator=generator)
    neg_sel = _smallest(neg_keys, negative, num_samples, num_samples - n_pos)
    return pos_sel, neg_sel


def _smallest(keys, mask, k, limit):
    """mask & (rank among the masked elements by ascending key < limit), with
    limit <= k (an int or an [N, 1] tensor): a top-k selection of the k
    smallest masked keys instead of a full sort of every row (a row is
    268,569 anchors in the RPN loss)."""
    N, P = keys.shape
    k = min(int(k), P)
    sel = torch.zeros_like(mask)
    if k <= 0:
        return sel
    if keys.is_cuda and k <= ops.TOPK_MAX_K:
        # the HIP segmented radix select (one segment per row) on -key: the k
        # largest of -key are the k smallest keys, ascending; unmasked -> -2
        neg = torch.where(mask, -keys, torch.full_like(keys, -2.0))
        start = torch.arange(N, device=keys.device, dtype=torch.int64) * P
        vals, idx, _ = ops.topk_segments(neg.reshape(-1), start,
                                         torch.full((N,), P, dtype=torch.int32,
                                                    device=keys.device), k, P)
        take = (torch.arange(k, device=keys.device)[None, :] < limit) & (vals > -2.0)
        return sel.scatter_(1, idx.long(), take)
    # beyond the HIP select's capacity (batch sizes above 8192 per image, e.g.
    # every anchor sampled) or off the GPU: a STABLE ascending sort, so tied
    # keys go to the lowest index first — the HIP select's tie rule (topk's
    # order among ties is unspecified)
    kk = torch.where(mask, keys, torch.full_like(keys, 2.0))
    vals, idx = torch.sort(kk, dim=1, stable=True)
    vals, idx = vals[:, :k], idx[:, :k]
    take = (torch.arange(k, device=keys.device)[None, :] < limit) & (vals < 2.0)
    return sel.scatter_(1, idx, take)
