"""RetinaNetHead (lib/modeling/single_stage_heads/retinanet.py:60-450).

Box tower: NUM_CONVS x (3x3 conv + ReLU) per branch + cls_score / bbox_pred
3x3 convs, all on the MFMA conv kernel.  Inference: d2mi_retinanet_inference —
per level sigmoid + exact top-k(min(1000, HWA)) over up to 12.1 M scores, score
threshold, decode of the chosen anchors with MODEL.RPN.BBOX_REG_WEIGHTS (as the
reference, retinanet.py:87), class-offset NMS, pad to DETECTIONS_PER_IMAGE.
Training (retinanet.py:147-283): IoU(valid GT, every anchor) + Matcher
(IOU_THRESHOLDS 0.4 / 0.5, low-quality matches) on the fused HIP matcher,
then sigmoid focal loss over every non-ignored anchor x class and smooth-L1
of the foreground deltas in one fused HIP pass over the head's per-level
outputs (d2mi_retina_loss_fwd / _bwd), both divided by the EMA of the
foreground count (the non-trainable loss_normalizer, momentum 0.9, init 100,
updated on the device before it divides: no host synchronisation)."""
import math

import torch

from ...layers import Conv2D, Layer, Sequential
from ...layers import initializers as init
from ...layers import ops
from ...structures import BoxList
from ...utils.arg_scope import arg_scope
from ..anchor_generator import build_anchor_generator
from ...layers.loss import sigmoid_focal_loss, smooth_l1_loss
from ..box_regression import Box2BoxTransform
from ..matcher import Matcher, match_boxes
from .build import SINGLE_STAGE_HEADS_REGISTRY


# the fused HIP losses on the GPU (False: the tensor formulation; tests compare)
FUSED_LOSSES = True


def _world():
    d = torch.distributed
    return d.get_world_size() if d.is_available() and d.is_initialized() else 1


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
        # training (retinanet.py:70-108)
        self.focal_loss_alpha = r.FOCAL_LOSS_ALPHA
        self.focal_loss_gamma = r.FOCAL_LOSS_GAMMA
        self.smooth_l1_loss_beta = r.SMOOTH_L1_LOSS_BETA
        s = cfg.MODEL.SINGLE_STAGE_HEAD
        self.matcher = Matcher(s.IOU_THRESHOLDS, s.IOU_LABELS, allow_low_quality_matches=True)
        self.register_buffer("loss_normalizer", torch.tensor(100.0))
        self.loss_normalizer_momentum = 0.9

    def call(self, images, features, targets=None):
        feats = [features[f] for f in self.in_features]
        box_cls, box_delta = self.head(feats)
        if self.training:
            if targets is None:
                raise ValueError("RetinaNet training needs targets")
            return None, self.losses(feats, box_cls, box_delta, targets)
        return self.inference(box_cls, box_delta), {}

    def _all_anchors(self, feats):
        """Level-major concatenation of the grid anchors (box_list_ops.concatenate
        of anchor_generator(features), retinanet.py:232), cached per grid."""
        key = tuple((f.shape[1], f.shape[2]) for f in feats) + (str(feats[0].device),)
        if getattr(self, "_anchor_key", None) != key:
            grids = [(f.shape[1], f.shape[2]) for f in feats]
            self._anchors = torch.cat(self.anchor_generator.grid_anchors(grids, feats[0].device))
            self._anchor_key = key
        return self._anchors

    def losses(self, feats, box_cls, box_delta, gt):
        """get_ground_truth + losses (retinanet.py:147-283) on dense [N, R]
        anchor rows: the GT matched against are the valid ones
        (boolean_mask(is_valid)); labels 1 -> the matched GT's class, 0 -> K
        (background), -1 -> ignored; the two sums over the whole batch are
        divided by the updated loss-normaliser EMA of max(1, #foreground)."""
        anchors = self._all_anchors(feats)
        gt_boxes, valid = gt["gt_boxes"], gt["is_valid"].bool()
        gt_classes = gt["gt_classes"]
        matches, labels = match_boxes(self.matcher, gt_boxes, valid, anchors)
        K = self.num_classes
        A = self.anchor_generator.num_cell_anchors[0]
        # the fused kernels read the logits as float4 class quads (K % 4 == 0,
        # e.g. COCO's 80); any other class count takes the tensor formulation
        if anchors.is_cuda and FUSED_LOSSES and K % 4 == 0:
            cls_sum, box_sum = ops.retina_loss(
                box_cls, box_delta, anchors, gt_boxes, gt_classes, matches, labels, K, A,
                self.focal_loss_alpha, self.focal_loss_gamma, self.smooth_l1_loss_beta,
                self.box2box_transform.weights)
        else:
            cls_sum, box_sum = self._losses_dense(box_cls, box_delta, anchors, gt_boxes,
                                                  gt_classes, matches, labels)
        with torch.no_grad():
            # moving_averages.assign_moving_average(zero_debias=False):
            # v -= (v - value) * (1 - momentum), value = max(1, #foreground)
            nfg = (labels == 1).sum().to(torch.float32).clamp(min=1.0)
            world = _world()
            if world > 1:
                # one normaliser for every replica (the reference's single
                # shared variable): the mean of the ranks' max(1, #fg), so the
                # replicas scale their losses alike and stay in sync
                torch.distributed.all_reduce(nfg)
                nfg = nfg / world
            v = self.loss_normalizer
            v.sub_((v - nfg) * (1.0 - self.loss_normalizer_momentum))
        norm = self.loss_normalizer.clone()  # (the next step's update stays out of this graph)
        return {"loss_cls": cls_sum / norm, "loss_box_reg": box_sum / norm}

    def _losses_dense(self, box_cls, box_delta, anchors, gt_boxes, gt_classes, matches, labels):
        """The tensor formulation of the two sums (CPU, and the tests'
        reference for the fused kernel): reshape_to_N_HWA_K + concat, the
        one-hot targets of the valid anchors, sigmoid_focal_loss "sum", and
        smooth_l1_loss "sum" of the foreground rows (retinanet.py:160-198)."""
        N, K = box_cls[0].shape[0], self.num_classes
        cls = torch.cat([c.reshape(N, -1, K) for c in box_cls], 1)
        dl = torch.cat([d.reshape(N, -1, 4) for d in box_delta], 1)
        gcls = torch.gather(gt_classes.to(torch.int64), 1, matches)
        tgt = torch.where(labels == 1, gcls, torch.where(labels == 0, torch.full_like(gcls, K),
                                                         torch.full_like(gcls, -1)))
        valid, fg = tgt >= 0, labels == 1
        onehot = torch.nn.functional.one_hot(tgt.clamp(min=0), K + 1)[..., :K].to(cls.dtype)
        focal = sigmoid_focal_loss(predictions=cls, targets=onehot, alpha=self.focal_loss_alpha,
                                   gamma=self.focal_loss_gamma)
        cls_sum = torch.where(valid[..., None], focal, torch.zeros_like(focal)).sum()
        gtb = torch.gather(gt_boxes, 1, matches[..., None].expand(-1, -1, 4))
        src = anchors[None].expand(N, -1, -1).reshape(-1, 4)
        target = self.box2box_transform.get_deltas(src, gtb.reshape(-1, 4)).reshape(N, -1, 4)
        l1 = smooth_l1_loss(labels=target, predictions=dl, beta=self.smooth_l1_loss_beta)
        box_sum = torch.where(fg[..., None], l1, torch.zeros_like(l1)).sum()
        return cls_sum, box_sum

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
