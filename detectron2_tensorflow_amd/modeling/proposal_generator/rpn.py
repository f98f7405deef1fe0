"""RPN (lib/modeling/proposal_generator/rpn.py:31-195, rpn_outputs.py:29-132, :403-440).

Head: shared 3x3 conv + ReLU and the objectness / anchor-delta 1x1 convs, all
on the MFMA conv kernel (the two 1x1s run as ONE 256 -> A + 4A GEMM whose
output is split).  Proposals: d2mi_rpn_proposals — per (image, level) exact
top-k of the logits, decode of the selected anchors only, clip, prune, per
level NMS, per-image top-k(post) and padding — in one fixed launch sequence.
"""
import torch

from ...layers import Conv2D, Layer
from ...layers import initializers as init
from ...layers import ops
from ...structures import BoxList
from ...utils.arg_scope import arg_scope
from ...utils.registry import Registry
from ..anchor_generator import build_anchor_generator
from ..box_regression import Box2BoxTransform
from .build import PROPOSAL_GENERATOR_REGISTRY

RPN_HEAD_REGISTRY = Registry("RPN_HEAD")


def build_rpn_head(cfg, input_shape, **kwargs):
    return RPN_HEAD_REGISTRY.get(cfg.MODEL.RPN.HEAD_NAME)(cfg, input_shape, **kwargs)


@RPN_HEAD_REGISTRY.register()
class StandardRPNHead(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        in_channels = {s.channels for s in input_shape}
        assert len(in_channels) == 1, "Each level must have the same channel!"
        in_channels = in_channels.pop()
        ag = build_anchor_generator(cfg, input_shape)
        A = set(ag.num_cell_anchors)
        assert len(A) == 1, "Each level must have the same number of cell anchors"
        self.A = A.pop()
        self.box_dim = ag.box_dim
        self.conv = Conv2D(in_channels, in_channels, 3, stride=1, activation="relu", scope="share")
        self.objectness_logits = Conv2D(in_channels, self.A, 1, stride=1, scope="objectness_logits")
        self.anchor_deltas = Conv2D(in_channels, self.A * self.box_dim, 1, stride=1,
                                    scope="anchor_deltas")
        self._fused = None
        self._fused_key = None

    def _fused_1x1(self):
        wo, wd = self.objectness_logits.weights, self.anchor_deltas.weights
        key = (wo._version, wd._version, wo.data_ptr(), wd.data_ptr())
        if self._fused is None or self._fused_key != key:
            w = torch.cat([wo.detach(), wd.detach()], dim=3)
            b = torch.cat([self.objectness_logits.bias.detach(), self.anchor_deltas.bias.detach()])
            self._fused = (ops.pack_conv_weights(w), b.contiguous())
            self._fused_key = key
        return self._fused

    def call(self, features):
        rpn_features, logits, deltas = [], [], []
        fuse = (not torch.is_grad_enabled()) and features[0].is_cuda
        for x in features:
            share = self.conv(x)
            rpn_features.append(share)
            if fuse:
                wp, b = self._fused_1x1()
                y = ops.conv2d_nhwc(share, wp, b)
                logits.append(y[..., : self.A].contiguous())
                deltas.append(y[..., self.A:].contiguous())
            else:
                logits.append(self.objectness_logits(share))
                deltas.append(self.anchor_deltas(share))
        return rpn_features, logits, deltas


@PROPOSAL_GENERATOR_REGISTRY.register()
class RPN(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        r = cfg.MODEL.RPN
        self.min_box_side_len = cfg.MODEL.PROPOSAL_GENERATOR.MIN_SIZE
        self.in_features = list(r.IN_FEATURES)
        self.nms_thresh = r.NMS_THRESH
        self.batch_size_per_image = r.BATCH_SIZE_PER_IMAGE
        self.positive_fraction = r.POSITIVE_FRACTION
        self.smooth_l1_beta = r.SMOOTH_L1_BETA
        self.loss_weight = r.LOSS_WEIGHT
        self.pre_nms_topk = {True: r.PRE_NMS_TOPK_TRAIN, False: r.PRE_NMS_TOPK_TEST}
        self.post_nms_topk = {True: r.POST_NMS_TOPK_TRAIN, False: r.POST_NMS_TOPK_TEST}
        self.boundary_threshold = r.BOUNDARY_THRESH
        shapes = [input_shape[f] for f in self.in_features]
        self.anchor_generator = build_anchor_generator(cfg, shapes)
        self.box2box_transform = Box2BoxTransform(weights=r.BBOX_REG_WEIGHTS)
        with arg_scope([Conv2D], weights_initializer=init.random_normal(0.01)):
            self.rpn_head = build_rpn_head(cfg, shapes, scope="rpn_head")

    def call(self, images, features, gt_instances=None):
        feats = [features[f] for f in self.in_features]
        rpn_features, logits, deltas = self.rpn_head(feats)
        if self.training:
            raise NotImplementedError("RPN training losses (matcher/sampler) are a later round "
                                      "(SURVEY.md section 8f, F2)")
        losses = {}
        boxes, scores, valid = ops.rpn_proposals(
            logits, deltas, self.anchor_generator.strides, self.anchor_generator.cell_anchors,
            images.image_shapes, self.pre_nms_topk[self.training],
            self.post_nms_topk[self.training], self.nms_thresh, float(self.min_box_side_len),
            self.box2box_transform.weights, self.box2box_transform.scale_clamp)
        proposals = BoxList(boxes)
        proposals.add_field("objectness_logits", scores)
        proposals.add_field("is_valid", valid)
        proposals.set_tracking("image_shape", images.image_shapes)
        return proposals, losses, dict(zip(self.in_features, rpn_features))
