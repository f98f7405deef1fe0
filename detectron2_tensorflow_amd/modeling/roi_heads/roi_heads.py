"""ROIHeads / StandardROIHeads (lib/modeling/roi_heads/roi_heads.py:66-605).

Dense, synchronisation-free layout: the RPN hands over [N, P] proposals with
an is_valid mask; every slot is pooled (invalid slots pool a zero box and are
dropped by the fused Fast R-CNN post-processing through roi_slot = -1), so
the box branch needs no tf.where / host round trip.  The mask branch pools
the [N, max_det] detections the same way and zeroes invalid rows — the
values the reference's SparseBoxList.to_dense produces.
"""
import torch

from ...layers import ShapeSpec, ops
from ...structures import BoxList
from ...utils import capture, host_sync
from ...utils.registry import Registry
from ..box_regression import Box2BoxTransform
from ..poolers import ROIPooler
from .box_head import build_box_head
from ..matcher import Matcher, match_boxes, subsample_labels
from .fast_rcnn import FastRCNNOutputLayers, fast_rcnn_inference, fast_rcnn_losses
from .mask_head import build_mask_head, mask_rcnn_inference, mask_rcnn_loss

from ...layers import Layer


# Per-step constant index tensors (image id of each row, per-image bases),
# cached per shape and device: read-only, so one tensor serves every step
# (two launches each fewer per use).
_INDEX_CACHE = {}


def _cached_index(kind, n, m, device):
    key = (kind, int(n), int(m), str(device))
    t = _INDEX_CACHE.get(key)
    if t is None:
        if len(_INDEX_CACHE) > 256:
            _INDEX_CACHE.clear()
        if kind == "img":  # arange(n).repeat_interleave(m), int32
            t = torch.arange(n, dtype=torch.int32, device=device).repeat_interleave(m)
        elif kind == "slot":  # arange(m).repeat(n), int32
            t = torch.arange(m, dtype=torch.int32, device=device).repeat(n)
        else:  # "base": arange(n)[:, None] * m, int64
            t = torch.arange(n, device=device)[:, None] * m
        # (made inside a hipGraph capture, the tensor holds its values only
        # once that graph has replayed: not cached for anything else)
        if not capture.capturing():
            _INDEX_CACHE[key] = t
    return t

ROI_HEADS_REGISTRY = Registry("ROI_HEADS")

# GPU: the sampled ROI batch in fg-first order straight from the fused
# sampler (d2mi_subsample order output) instead of a key sort (A/B switch)
FUSED_ORDER = True


def build_roi_heads(cfg, input_shape, **kwargs):
    return ROI_HEADS_REGISTRY.get(cfg.MODEL.ROI_HEADS.NAME)(cfg, input_shape, **kwargs)


class ROIHeads(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        h = cfg.MODEL.ROI_HEADS
        self.batch_size_per_image = h.BATCH_SIZE_PER_IMAGE
        self.positive_sample_fraction = h.POSITIVE_FRACTION
        self.test_score_thresh = h.SCORE_THRESH_TEST
        self.test_nms_thresh = h.NMS_THRESH_TEST
        self.test_nms_cls_agnostic = h.NMS_CLS_AGNOSTIC
        self.test_detections_per_img = cfg.TEST.DETECTIONS_PER_IMAGE
        self.in_features = list(h.IN_FEATURES)
        self.num_classes = h.NUM_CLASSES
        self.proposal_append_gt = h.PROPOSAL_APPEND_GT
        self.feature_strides = {k: v.stride for k, v in input_shape.items()}
        self.feature_channels = {k: v.channels for k, v in input_shape.items()}
        self.cls_agnostic_bbox_reg = cfg.MODEL.ROI_BOX_HEAD.CLS_AGNOSTIC_BBOX_REG
        self.smooth_l1_beta = cfg.MODEL.ROI_BOX_HEAD.SMOOTH_L1_BETA
        self.box2box_transform = Box2BoxTransform(weights=cfg.MODEL.ROI_BOX_HEAD.BBOX_REG_WEIGHTS)
        self.proposal_matcher = Matcher(h.IOU_THRESHOLDS, h.IOU_LABELS,
                                        allow_low_quality_matches=False)

    def label_and_sample_proposals(self, proposals, targets):
        """roi_heads.py:100-232 batched: append GT (proposal_utils.py:7-60), match
        (crowd -> ignore bg, difficult -> ignore bg above the threshold), gt_classes
        (fg class / bg = NUM_CLASSES / -1), subsample, fg-first order, pad.
        Returns a dict of [N, S] tensors: boxes, gt_classes, gt_boxes, gt_index
        (matched GT row), is_valid."""
        boxes = proposals.boxes
        pvalid = proposals.get_field("is_valid")
        gt_boxes = targets["gt_boxes"]
        gvalid = targets["is_valid"].bool()
        N, G = gvalid.shape
        zeros = torch.zeros_like(gvalid)
        crowd = targets.get("gt_is_crowd", zeros).bool()
        difficult = targets.get("gt_difficult", zeros).bool()
        if self.proposal_append_gt:
            boxes = torch.cat([boxes, gt_boxes.to(boxes.dtype)], dim=1)
            pvalid = torch.cat([pvalid, gvalid], dim=1)
        M = boxes.shape[1]
        # (matched against the valid GT that are neither crowd nor difficult)
        matches, labels = match_boxes(self.proposal_matcher, gt_boxes, gvalid, boxes,
                                      crowd=crowd, difficult=difficult)
        K = self.num_classes
        S = self.batch_size_per_image
        if boxes.is_cuda and FUSED_ORDER and ops.FUSED_SAMPLE_TAKE:
            # two launches for the glue (d2mi_roi_gt_classes, d2mi_roi_sample_take),
            # the mask branch's fg-first inputs and foreground count included
            gt_classes = ops.roi_gt_classes(labels, matches, targets["gt_classes"], pvalid, K)
            _, _, order, valid = subsample_labels(gt_classes, S, self.positive_sample_fraction, K,
                                                  order_slots=S)
            F_ = (int(S * self.positive_sample_fraction)
                  if getattr(self, "mask_on", False) and getattr(self, "mask_compact_rows", False)
                  else 0)
            sampled, mprep = ops.roi_sample_take(order, valid, boxes, gt_classes, matches,
                                                 gt_boxes, K, F_)
            if mprep is not None:
                sampled["_mask_prep"] = mprep
            return sampled
        gcls = torch.gather(targets["gt_classes"].long(), 1, matches)
        # label 1 -> the matched GT class, 0 -> background K, -1 -> ignored;
        # invalid proposal slots -> -1
        gt_classes = torch.where(labels == 1, gcls, torch.where(labels == 0, K, labels))
        gt_classes = torch.where(pvalid, gt_classes, -1)
        if boxes.is_cuda and FUSED_ORDER:
            # fused: the sampled rows come back in fg-first, index order
            _, _, order, valid = subsample_labels(gt_classes, S, self.positive_sample_fraction, K,
                                                  order_slots=S)
        else:
            pos, neg = subsample_labels(gt_classes, S, self.positive_sample_fraction, K)
            ar = torch.arange(M, device=boxes.device)
            key = torch.where(pos, 0, torch.where(neg, 1, 2)) * M + ar
            if M < S:
                key = torch.cat([key, torch.full((N, S - M), 3 * M, dtype=key.dtype,
                                                 device=key.device)], dim=1)
            key = key.sort(dim=1).values[:, :S]
            valid = key < 2 * M
            order = torch.where(valid, key % M, torch.zeros_like(key))
        take = lambda t: torch.gather(t, 1, order)
        take4 = lambda t: torch.gather(t, 1, order[..., None].expand(-1, -1, 4))
        gidx = take(matches)
        return {"boxes": take4(boxes), "gt_classes": take(gt_classes), "gt_index": gidx,
                "gt_boxes": torch.gather(gt_boxes, 1, gidx[..., None].expand(-1, -1, 4)),
                "is_valid": valid}


class DeferredMaskLoss:
    """The training mask loss of a StandardROIHeads forward, not yet run:
    the foreground count is known only on the device (``count``), and the
    compacted mask branch's row count depends on it.  A step captured into
    hipGraphs (engine/graphed.py) replays the forward up to here, reads
    ``count`` once, and replays the mask branch + backward graph captured for
    that row count (``compute(rows)``, run once per distinct row count at
    capture time).  The eager trainer never sees one (defer_mask_loss False)."""

    def __init__(self, heads, feats, sampled, targets, share, fg, prep=None, count=None):
        self.heads, self.feats, self.sampled, self.targets = heads, feats, sampled, targets
        self.share, self.fg, self.prep = share, fg, prep
        self.count = fg.sum() if count is None else count
        self.slots = fg.numel()

    def rows_for(self, nfg):
        return self.heads.mask_rows(int(nfg), self.slots)

    def compute(self, rows):
        return self.heads._mask_loss(self.feats, self.sampled, self.targets, self.share, None,
                                     self.fg, rows=rows, prep=self.prep)


@ROI_HEADS_REGISTRY.register()
class StandardROIHeads(ROIHeads):
    MASK_ROW_BUCKET = 32
    # the mask branch's fg-first ordering and per-slot gathers issued before
    # the foreground-count read, so less host work follows it
    MASK_PREP_EARLY = True

    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(cfg, input_shape, **kwargs)
        self._init_box_head(cfg)
        self._init_mask_head(cfg)

    def _init_box_head(self, cfg):
        b = cfg.MODEL.ROI_BOX_HEAD
        scales = tuple(1.0 / self.feature_strides[k] for k in self.in_features)
        chans = {self.feature_channels[f] for f in self.in_features}
        assert len(chans) == 1, chans
        c = chans.pop()
        self.box_pooler = ROIPooler(b.POOLER_RESOLUTION, scales, b.POOLER_SAMPLING_RATIO,
                                    b.POOLER_TYPE)
        self.box_head = build_box_head(cfg, ShapeSpec(channels=c, height=b.POOLER_RESOLUTION,
                                                      width=b.POOLER_RESOLUTION), scope="box_head")
        self.box_predictor = FastRCNNOutputLayers(self.box_head.output_size, self.num_classes,
                                                  self.cls_agnostic_bbox_reg, scope="box_predictor")

    def _init_mask_head(self, cfg):
        self.mask_on = cfg.MODEL.MASK_ON
        if not self.mask_on:
            return
        m = cfg.MODEL.ROI_MASK_HEAD
        self.use_mini_masks = cfg.TRANSFORM.RESIZE.USE_MINI_MASKS
        # True: mask head on the foreground rows only, like the reference (one
        # host sync per step); False: fixed [N, S*POSITIVE_FRACTION] rows with
        # a validity mask (no host sync, capturable).
        self.mask_compact_rows = True
        # True (set by engine.graphed.GraphedTrainer): the training forward
        # returns a DeferredMaskLoss instead of reading the foreground count
        self.defer_mask_loss = False
        self.last_mask_rows = None
        scales = tuple(1.0 / self.feature_strides[k] for k in self.in_features)
        c = [self.feature_channels[f] for f in self.in_features][0]
        self.mask_pooler = ROIPooler(m.POOLER_RESOLUTION, scales, m.POOLER_SAMPLING_RATIO,
                                     m.POOLER_TYPE)
        self.mask_head = build_mask_head(cfg, ShapeSpec(channels=c, width=m.POOLER_RESOLUTION,
                                                        height=m.POOLER_RESOLUTION), scope="mask_head")

    def call(self, images, features, proposals, targets=None):
        feats = [features[f] for f in self.in_features]
        if self.training:
            if targets is None:
                raise ValueError("ROI-head training needs targets")
            sampled = self.label_and_sample_proposals(proposals, targets)
            # the box and mask poolers read the same p2..p5: one gradient map
            # set for both backwards (ops._RoIAlignFn grad_share)
            share = {} if self.mask_on else None
            # the mask branch's foreground count is read while the box branch
            # is enqueued (the device never idles at the read)
            pending = None
            # (d2mi_roi_sample_take: the mask branch's fg-first inputs, fg and
            # the foreground count made with the sampled rows)
            fused = sampled.pop("_mask_prep", None)
            fg = (fused[1] if fused is not None
                  else self._mask_fg(sampled) if self.mask_on else None)  # (once per step)
            count = fused[2] if fused is not None else None
            defer = self.mask_on and self.mask_compact_rows and self.defer_mask_loss
            prep = None
            if self.mask_on and self.mask_compact_rows:
                if not defer:
                    pending = host_sync.start_read(count if count is not None else fg.sum())
                # (deferred too, r5: in a replayed step these small gathers are
                # issued inside graph A, under the box branch's kernels, not at
                # graph B's head where the host's per-node submission outran them)
                if fused is not None:
                    gm = targets["gt_masks"]
                    prep = (fused[0], gm.reshape(gm.shape[0] * gm.shape[1], *gm.shape[2:]), fg)
                elif self.MASK_PREP_EARLY:
                    prep = self._mask_prep(sampled, targets, fg)
            losses = self._box_losses(feats, sampled, share)
            if defer:
                losses["loss_mask"] = DeferredMaskLoss(self, feats, sampled, targets, share, fg,
                                                       prep, count)
            elif self.mask_on:
                losses["loss_mask"] = self._mask_loss(feats, sampled, targets, share, pending, fg,
                                                      prep=prep)
            return sampled, losses
        pred = self._forward_box(feats, proposals, images.image_shapes)
        pred = self.forward_with_given_boxes(features, pred)
        return pred, {}

    def _forward_box(self, feats, proposals, image_shapes):
        boxes = proposals.boxes
        valid = proposals.get_field("is_valid")
        N, P = valid.shape
        dev = boxes.device
        img = _cached_index("img", N, P, dev)
        slot = _cached_index("slot", N, P, dev)
        slot = torch.where(valid.reshape(-1), slot, torch.full_like(slot, -1))
        x = self.box_pooler.pool(feats, boxes.reshape(-1, 4), img)
        x = self.box_head(x)
        logits, deltas = self.box_predictor(x)
        ob, os_, oc, ov, _ = fast_rcnn_inference(
            logits, deltas, boxes.reshape(-1, 4), img, slot, N, P, image_shapes,
            self.box2box_transform, self.test_score_thresh, self.test_nms_thresh,
            self.test_detections_per_img, self.test_nms_cls_agnostic)
        res = BoxList(ob)
        res.add_field("scores", os_)
        res.add_field("pred_classes", oc)
        res.add_field("is_valid", ov)
        res.set_tracking("image_shape", image_shapes)
        return res

    def _box_losses(self, feats, sampled, grad_share=None):
        boxes = sampled["boxes"]
        N, S = boxes.shape[:2]
        img = _cached_index("img", N, S, boxes.device)
        x = self.box_pooler.pool(feats, boxes.reshape(-1, 4).contiguous(), img,
                                 grad_share=grad_share)
        logits, deltas = self.box_predictor(self.box_head(x))
        return fast_rcnn_losses(logits, deltas, boxes.reshape(-1, 4), sampled["gt_classes"].reshape(-1),
                                sampled["gt_boxes"].reshape(-1, 4), sampled["is_valid"].reshape(-1),
                                self.box2box_transform, self.smooth_l1_beta)

    def _mask_fg(self, sampled):
        """Foreground flags of the first int(S * POSITIVE_FRACTION) slots per image:
        valid and not background.  (A sampled slot is a positive, class in
        [0, K), or a negative, class K -- the ignored -1 rows are never
        sampled -- so `class < K` is the reference's `!= -1 and != bg` there.)"""
        F_ = int(self.batch_size_per_image * self.positive_sample_fraction)
        return (sampled["is_valid"][:, :F_]
                & (sampled["gt_classes"][:, :F_] < self.num_classes)).reshape(-1)

    def mask_rows(self, nfg, slots):
        """Rows the compacted mask branch runs for nfg foreground proposals out
        of ``slots``: nfg rounded up to a multiple of MASK_ROW_BUCKET (at least
        one bucket, at most every slot) -- a handful of distinct shapes."""
        b = self.MASK_ROW_BUCKET
        return min(slots, max(b, -(-nfg // b) * b))

    def _mask_prep(self, sampled, targets, fg=None):
        """The mask branch's per-slot inputs over the first int(S *
        POSITIVE_FRACTION) slots per image, and (compact rows) the slots in
        fg-first order -- everything that does not need the foreground count,
        so the host issues it before the count's read."""
        F_ = int(self.batch_size_per_image * self.positive_sample_fraction)
        boxes = sampled["boxes"][:, :F_].reshape(-1, 4)
        N = sampled["boxes"].shape[0]
        dev = boxes.device
        cls = sampled["gt_classes"][:, :F_].reshape(-1)
        fg = self._mask_fg(sampled) if fg is None else fg
        img = _cached_index("img", N, F_, dev)
        gm = targets["gt_masks"]
        G = gm.shape[1]
        mind = (sampled["gt_index"][:, :F_] + _cached_index("base", N, G, dev)).reshape(-1)
        gt_boxes = sampled["gt_boxes"][:, :F_].reshape(-1, 4)
        ts = (boxes, cls, fg, img, mind, gt_boxes)
        if self.mask_compact_rows:
            # fg rows first, each group in index order (a stable sort of ~fg);
            # the count only decides how many of them run (a view)
            order = torch.argsort((~fg).to(torch.uint8), stable=True)
            ts = tuple(t[order] for t in ts)
        return ts, gm.reshape(N * G, *gm.shape[2:]), fg

    def _mask_loss(self, feats, sampled, targets, grad_share=None, pending=None, fg=None,
                   rows=None, prep=None):
        """_forward_mask training branch (roi_heads.py:594-600) over the first
        int(S * POSITIVE_FRACTION) slots per image, which hold every sampled
        foreground proposal (select_foreground_proposals, roi_heads.py:35-62)."""
        ts, gm, fg_all = prep if prep is not None else self._mask_prep(sampled, targets, fg)
        if self.mask_compact_rows:
            # The reference runs the mask head on the foreground proposals only
            # (select_foreground_proposals, roi_heads.py:35-62 + :594-600).  One
            # host read of the foreground count; the rows are gathered fg-first
            # (image order kept) and padded to a multiple of MASK_ROW_BUCKET
            # with masked-out rows, which bounds the number of distinct shapes.
            # (rows given: a deferred mask loss, DeferredMaskLoss.compute)
            if rows is None:
                nfg = (host_sync.finish_read(pending) if pending is not None
                       else host_sync.read_ints(fg_all.sum()))[0]
                rows = self.mask_rows(nfg, fg_all.numel())
            R = rows
            ts = tuple(t[:R] for t in ts)
            self.last_mask_rows = R
        else:
            self.last_mask_rows = int(ts[0].shape[0])
        boxes, cls, fg, img, mind, gt_boxes = ts
        x = self.mask_pooler.pool(feats, boxes.contiguous(), img, grad_share=grad_share)
        _, logits = self.mask_head(x)
        return mask_rcnn_loss(logits, boxes, gt_boxes, cls, gm, mind, fg, self.use_mini_masks)

    def forward_with_given_boxes(self, features, instances, image_shape=None):
        assert not self.training
        assert instances.has_field("pred_classes")
        if not self.mask_on:
            return instances
        feats = [features[f] for f in self.in_features]
        boxes = instances.boxes
        N, D = boxes.shape[:2]
        img = _cached_index("img", N, D, boxes.device)
        x = self.mask_pooler.pool(feats, boxes.reshape(-1, 4), img)
        deconv, logits = self.mask_head(x)
        masks = mask_rcnn_inference(logits, instances.get_field("pred_classes").reshape(-1))
        valid = instances.get_field("is_valid").reshape(-1)
        masks = masks * valid[:, None, None].to(masks.dtype)
        instances.add_field("pred_masks", masks.reshape(N, D, *masks.shape[1:]))
        return instances
