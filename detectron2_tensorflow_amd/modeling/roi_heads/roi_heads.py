"""ROIHeads / StandardROIHeads (lib/modeling/roi_heads/roi_heads.py:66-605), inference.

Dense, synchronisation-free layout: the RPN hands over [N, P] proposals with
an is_valid mask; every slot is pooled (invalid slots pool a zero box and are
dropped by the fused Fast R-CNN post-processing through roi_slot = -1), so
the box branch needs no tf.where / host round trip.  The mask branch pools
the [N, max_det] detections the same way and zeroes invalid rows — the
values the reference's SparseBoxList.to_dense produces.
"""
import torch

from ...layers import ShapeSpec
from ...structures import BoxList
from ...utils.registry import Registry
from ..box_regression import Box2BoxTransform
from ..poolers import ROIPooler
from .box_head import build_box_head
from .fast_rcnn import FastRCNNOutputLayers, fast_rcnn_inference
from .mask_head import build_mask_head, mask_rcnn_inference

from ...layers import Layer

ROI_HEADS_REGISTRY = Registry("ROI_HEADS")


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


@ROI_HEADS_REGISTRY.register()
class StandardROIHeads(ROIHeads):
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
        scales = tuple(1.0 / self.feature_strides[k] for k in self.in_features)
        c = [self.feature_channels[f] for f in self.in_features][0]
        self.mask_pooler = ROIPooler(m.POOLER_RESOLUTION, scales, m.POOLER_SAMPLING_RATIO,
                                     m.POOLER_TYPE)
        self.mask_head = build_mask_head(cfg, ShapeSpec(channels=c, width=m.POOLER_RESOLUTION,
                                                        height=m.POOLER_RESOLUTION), scope="mask_head")

    def call(self, images, features, proposals, targets=None):
        if self.training:
            raise NotImplementedError("ROI-head training (label_and_sample_proposals, losses) is "
                                      "a later round (SURVEY.md section 8f, F2)")
        feats = [features[f] for f in self.in_features]
        pred = self._forward_box(feats, proposals, images.image_shapes)
        pred = self.forward_with_given_boxes(features, pred)
        return pred, {}

    def _forward_box(self, feats, proposals, image_shapes):
        boxes = proposals.boxes
        valid = proposals.get_field("is_valid")
        N, P = valid.shape
        dev = boxes.device
        img = torch.arange(N, dtype=torch.int32, device=dev).repeat_interleave(P)
        slot = torch.arange(P, dtype=torch.int32, device=dev).repeat(N)
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

    def forward_with_given_boxes(self, features, instances, image_shape=None):
        assert not self.training
        assert instances.has_field("pred_classes")
        if not self.mask_on:
            return instances
        feats = [features[f] for f in self.in_features]
        boxes = instances.boxes
        N, D = boxes.shape[:2]
        img = torch.arange(N, dtype=torch.int32, device=boxes.device).repeat_interleave(D)
        x = self.mask_pooler.pool(feats, boxes.reshape(-1, 4), img)
        deconv, logits = self.mask_head(x)
        masks = mask_rcnn_inference(logits, instances.get_field("pred_classes").reshape(-1))
        valid = instances.get_field("is_valid").reshape(-1)
        masks = masks * valid[:, None, None].to(masks.dtype)
        instances.add_field("pred_masks", masks.reshape(N, D, *masks.shape[1:]))
        return instances
