"""RetinaNetHead inference (lib/modeling/single_stage_heads/retinanet.py:60-450).

Box tower: NUM_CONVS x (3x3 conv + ReLU) per branch + cls_score / bbox_pred
3x3 convs, all on the MFMA conv kernel.  Inference: d2mi_retinanet_inference —
per level sigmoid + exact top-k(min(1000, HWA)) over up to 12.1 M scores, score
threshold, decode of the chosen anchors with MODEL.RPN.BBOX_REG_WEIGHTS (as the
reference, retinanet.py:87), class-offset NMS, pad to DETECTIONS_PER_IMAGE."""
import math

import torch

from ...layers import Conv2D, Layer, Sequential
from ...layers import initializers as init
from ...layers import ops
from ...structures import BoxList
from ...utils.arg_scope import arg_scope
from ..anchor_generator import build_anchor_generator
from ..box_regression import Box2BoxTransform
from .build import SINGLE_STAGE_HEADS_REGISTRY


class RetinaNetBoxTower(Layer):
    def __init__(self, cfg, input_shape, num_anchors, **kwargs):
        super().__init__(**kwargs)
        cin = input_shape[0].channels
        K = cfg.MODEL.SINGLE_STAGE_HEAD.NUM_CLASSES
        n = cfg.MODEL.RETINANET.NUM_CONVS
        prior = cfg.MODEL.RETINANET.PRIOR_PROB
        assert len(set(num_anchors)) == 1
        A = num_anchors[0]
        with arg_scope([Conv2D], kernel_size=3, stride=1, padding="SAME", activation="relu",
                       weights_initializer=init.random_normal(0.01)):
            cls, box = [], []
            for i in range(n):
                cls.append(Conv2D(cin, cin, scope=f"cls_subnet{2 * i}"))
                box.append(Conv2D(cin, cin, scope=f"bbox_subnet{2 * i}"))
            self.cls_layers = torch.nn.ModuleList(cls)
            self.box_layers = torch.nn.ModuleList(box)
            self.cls_subnet = Sequential(cls)
            self.bbox_subnet = Sequential(box)
            self.cls_score = Conv2D(cin, A * K, activation=None,
                                    bias_initializer=init.constant(-math.log((1 - prior) / prior)),
                                    scope="cls_score")
            self.bbox_pred = Conv2D(cin, A * 4, activation=None, scope="bbox_pred")

    def call(self, features):
        """Per level: cls_score(cls_subnet(f)), bbox_pred(bbox_subnet(f))
        (retinanet.py:110-145, variables shared across levels).  Each layer
        runs over all levels in one multi-level launch (Conv2D.call_levels)."""
        c, b = list(features), list(features)
        for layer in self.cls_layers:
            c = layer.call_levels(c)
        for layer in self.box_layers:
            b = layer.call_levels(b)
        return self.cls_score.call_levels(c), self.bbox_pred.call_levels(b)


@SINGLE_STAGE_HEADS_REGISTRY.register()
class RetinaNetHead(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        self.num_classes = cfg.MODEL.SINGLE_STAGE_HEAD.NUM_CLASSES
        self.in_features = list(cfg.MODEL.SINGLE_STAGE_HEAD.IN_FEATURES)
        r = cfg.MODEL.RETINANET
        self.score_threshold = r.SCORE_THRESH_TEST
        self.topk_candidates = r.TOPK_CANDIDATES_TEST
        self.nms_threshold = r.NMS_THRESH_TEST
        self.max_detections_per_image = cfg.TEST.DETECTIONS_PER_IMAGE
        shapes = [input_shape[f] for f in self.in_features]
        self.anchor_generator = build_anchor_generator(cfg, shapes)
        self.head = RetinaNetBoxTower(cfg, shapes, self.anchor_generator.num_cell_anchors, scope="head")
        self.box2box_transform = Box2BoxTransform(weights=cfg.MODEL.RPN.BBOX_REG_WEIGHTS)

    def call(self, images, features, targets=None):
        feats = [features[f] for f in self.in_features]
        box_cls, box_delta = self.head(feats)
        if self.training:
            raise NotImplementedError("RetinaNet training (focal loss, matcher) is a later round")
        return self.inference(box_cls, box_delta), {}

    def inference(self, box_cls, box_delta):
        ob, os_, oc, ov = ops.retinanet_inference(
            box_cls, box_delta, self.anchor_generator.strides, self.anchor_generator.cell_anchors,
            self.num_classes, self.topk_candidates, self.score_threshold, self.nms_threshold,
            self.max_detections_per_image, self.box2box_transform.weights,
            self.box2box_transform.scale_clamp)
        res = BoxList(ob)
        res.add_field("scores", os_)
        res.add_field("pred_classes", oc)
        res.add_field("is_valid", ov)
        return res
