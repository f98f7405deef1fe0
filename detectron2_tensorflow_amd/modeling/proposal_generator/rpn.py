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
from ...layers import handoff, ops
from ...layers.loss import smooth_l1_loss
from ..matcher import Matcher, match_boxes, subsample_labels
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
    # training: the fused head's outputs gathered into the RPNOutputs layout
    # in one launch (False: per-level slice copies + concatenation, A/B)
    CONCAT_OUT = True
    # True: the shared 3x3's weight / bias gradient accumulates over the FPN
    # levels in one buffer (the MFMA wgrad's reduce adds each level into it;
    # layers/convolutional.py:_wgrad_shared) -- autograd's per-level adds go
    ACC_CONV_LEVELS = True

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
        self._fused_pad = None

    def _fused_1x1(self):
        """The objectness (A) and anchor-delta (4A) 1x1 convs as ONE conv of
        A + 4A outputs, zero-padded to a multiple of 4 (15 -> 16): weights
        HWIO [1, 1, C, 16], their MFMA packing, and the bias [16]."""
        wo, wd = self.objectness_logits.weights, self.anchor_deltas.weights
        bo, bd = self.objectness_logits.bias, self.anchor_deltas.bias
        key = (wo._version, wd._version, bo._version, bd._version, wo.data_ptr(), wd.data_ptr())
        if self._fused is None or self._fused_key != key:
            n = wo.shape[3] + wd.shape[3]
            pad = (-n) % 4
            zp = self._fused_pad
            if zp is None or zp[0].shape[:3] != wo.shape[:3] or zp[0].shape[3] != pad \
                    or zp[0].device != wo.device:
                # the zero pad columns, made once (not two fills per step)
                zp = self._fused_pad = (wo.new_zeros(*wo.shape[:3], pad), bo.new_zeros(pad))
            w = torch.cat([wo.detach(), wd.detach(), zp[0]], dim=3)
            b = torch.cat([bo.detach(), bd.detach(), zp[1]])
            self._fused = (w.contiguous(), ops.pack_conv_weights(w), b.contiguous())
            self._fused_key = key
        return self._fused

    def call(self, features):
        rpn_features, logits, deltas = [], [], []
        fuse = features[0].is_cuda
        if fuse and not torch.is_grad_enabled() and len(features) <= 6:
            # inference: the shared 3x3 and the fused 16-wide 1x1 each as ONE
            # multi-level launch over p2..p6
            shares = self.conv.call_levels(list(features))
            w16, wp, b16 = self._fused_1x1()
            A, D = self.objectness_logits.weights.shape[3], self.anchor_deltas.weights.shape[3]
            for y in ops.conv2d_nhwc_levels(shares, wp, b16):
                logits.append(y[..., :A].contiguous())
                deltas.append(y[..., A:A + D].contiguous())
            return shares, logits, deltas
        # the fused 1x1's weight / bias gradient accumulates over the levels in
        # one buffer (each level's skinny wgrad adds into it; the last level
        # returns the sum): autograd's per-level adds and slices go away
        wacc = ({"n": len(features), "k": 0}
                if fuse and torch.is_grad_enabled() and _RPNHead1x1Fn.ACC_LEVELS else None)
        cacc = ({"n": len(features), "k": 0}
                if fuse and torch.is_grad_enabled() and StandardRPNHead.ACC_CONV_LEVELS else None)
        ys = []
        pairs = [getattr(x, "_d2mi_grad_pair", None) for x in features]
        for li, x in enumerate(features):
            # a level the ROI poolers also read hands its input gradient over
            # (GeneralizedRCNN tags them; the pair_grad protocol)
            share = self.conv(x, pair_grad=pairs[li], wacc=cacc)
            if fuse:
                # the fused 1x1 is the declared SOLE consumer of the 3x3's ReLU
                # output (its dgrad applies the ReLU mask, _RPNHead1x1Fn): the
                # features handed back are detached, so nothing else adds an
                # ungated gradient to it
                rpn_features.append(share.detach())
            else:
                rpn_features.append(share)
            if fuse:
                w16, wp, b16 = self._fused_1x1()
                ys.append(_RPNHead1x1Fn.apply(share, self.objectness_logits.weights,
                                              self.objectness_logits.bias,
                                              self.anchor_deltas.weights, self.anchor_deltas.bias,
                                              w16, wp, b16, wacc))
            else:
                logits.append(self.objectness_logits(share))
                deltas.append(self.anchor_deltas(share))
        if fuse and not StandardRPNHead.CONCAT_OUT:  # (A/B: per-level slice copies)
            A = self.objectness_logits.weights.shape[3]
            logits = [y[..., :A].contiguous() for y in ys]
            deltas = [y[..., A:5 * A].contiguous() for y in ys]
        elif fuse:
            # the RPNOutputs layout (rpn_outputs.py:346-357) straight from the
            # fused outputs, one launch each way (_RPNGatherFn); the per-level
            # logits / deltas handed on are views of it
            A = self.objectness_logits.weights.shape[3]
            pl, pd = _RPNGatherFn.apply(A, *ys)
            logits, deltas = _LevelViews(), _LevelViews()
            off = 0
            for y in ys:
                N, H, W, _ = y.shape
                logits.append(pl[:, off * A:(off + H * W) * A].view(N, H, W, A))
                deltas.append(pd[:, off * A:(off + H * W) * A].view(N, H, W, 4 * A))
                off += H * W
            logits.concat = deltas.concat = (pl, pd)
        return rpn_features, logits, deltas


class _LevelViews(list):
    """Per-level views of one concatenated [N, sum_l H_l W_l A] (x4) tensor;
    ``concat`` is that (logits, deltas) pair."""
    concat = None


class _RPNGatherFn(torch.autograd.Function):
    """The fused 1x1's per-level [N, H, W, 16] outputs -> (objectness logits
    [N, T*A], anchor deltas [N, T*A, 4]) in the level-major per-image layout
    of RPNOutputs (rpn_outputs.py:346-357), by d2mi_rpn_head_gather; backward
    = d2mi_rpn_head_scatter straight into the per-level 16-wide gradients
    (padding channel zero): no slice copies, concatenations or zero-fills."""

    @staticmethod
    def forward(ctx, A, *ys):
        ctx.A = A
        ctx.shapes = [tuple(y.shape) for y in ys]
        ctx.set_materialize_grads(False)
        return ops.rpn_head_gather(ys, A)

    @staticmethod
    def backward(ctx, g_logits, g_deltas):
        if g_logits is None and g_deltas is None:
            return (None,) * (1 + len(ctx.shapes))
        return (None, *ops.rpn_head_scatter(g_logits, g_deltas, ctx.shapes, ctx.A))


class _RPNHead1x1Fn(torch.autograd.Function):
    """Both RPN-head 1x1 convs (rpn.py:83-96) as one 16-wide conv on the MFMA
    kernel.  Backward: the two output gradients are concatenated (+ the zero
    pad column) into one [.., 16] gradient; the input gradient is ONE dgrad
    conv (instead of a dgrad per head + their sum), the weight and bias
    gradients one skinny X^T G pass (d2mi_wgrad_skinny) sliced per head.  The
    input gradient leaves through the dgrad's ReLU gate (share > 0) when share
    is a fused-ReLU conv output, which then skips its threshold_backward (the
    sole-consumer protocol of layers/convolutional.py:_ConvMFMAFn)."""
    GATE = True  # False: leave the ReLU backward to the 3x3 conv (tests)
    # True: the levels of one forward share a weight-gradient accumulator
    # (wacc: {"n": levels, "k": done}); every level but the last returns no
    # weight gradient, the last one the in-order sum -- autograd's
    # ((g1 + g2) + g3) ... of the per-level gradients, without its adds
    ACC_LEVELS = True
    # True: the levels' skinny wgrads as ONE multi-level launch pair at the
    # last level's backward (d2mi_wgrad_skinny_levels, bit-identical sums)
    LEVELS_ONE_LAUNCH = True

    @staticmethod
    def forward(ctx, share, wo, bo, wd, bd, w16, wp, b16, wacc=None):
        y = ops.conv2d_nhwc(share, wp, b16)
        A, D = wo.shape[3], wd.shape[3]
        ctx.save_for_backward(share, w16)
        ctx.relu_info = getattr(share, "_d2mi_relu_info", None) if _RPNHead1x1Fn.GATE else None
        ctx.set_materialize_grads(False)  # a missing gradient is a zero one below
        ctx.dims = (A, D, y.shape[-1])
        ctx.wacc = wacc
        return y  # [.., 16]: A logits, 4A deltas, zero padding (_RPNGatherFn splits it)

    @staticmethod
    def backward(ctx, g16):
        share, w16 = ctx.saved_tensors
        A, D, C16 = ctx.dims
        if g16 is None:
            g16 = share.new_zeros(*share.shape[:-1], C16)
        gx = None
        if ctx.needs_input_grad[0]:
            # 1x1 stride-1 dgrad: the forward weights' HWIO [1, 1, C, 16] is
            # the packed layout of the transposed conv
            info = ctx.relu_info
            if info is not None and share.shape[-1] % 4 == 0:
                gx = ops.conv2d_nhwc(g16, w16, None, 1, (0, 0), relu_gate=share)
                info["masked"] = True
            else:
                gx = ops.conv2d_nhwc(g16, w16, None, 1, (0, 0))
        acc = ctx.wacc
        if acc is not None:
            acc["k"] += 1
            if acc["k"] == 1:
                # every level's backward must run in this pass: otherwise the
                # weight gradient (returned by the last level) never leaves
                # and a stale buffer would poison a later backward
                handoff.expect_complete(acc, lambda a: a["k"] == 0,
                                        lambda a: (a.pop("buf", None), a.pop("lv", None),
                                                   a.__setitem__("k", 0)),
                                        "RPN head 1x1 weight-gradient levels")
            if _RPNHead1x1Fn.LEVELS_ONE_LAUNCH:
                # the levels' (input, gradient) pairs in backward order, one
                # multi-level skinny wgrad at the last (the same sums)
                acc.setdefault("lv", []).append((share, g16))
            else:
                acc["buf"] = ops.wgrad_skinny(share, g16, with_bias=True,
                                              accumulate_into=acc.get("buf"))
            if acc["k"] < acc["n"]:
                return gx, None, None, None, None, None, None, None, None
            if _RPNHead1x1Fn.LEVELS_ONE_LAUNCH:
                lv = acc.pop("lv")
                if len(lv) <= 8 and all(ops.skinny_levels_ok(x) for x, _ in lv):
                    gw, gb = ops.wgrad_skinny_levels([x for x, _ in lv], [g for _, g in lv])
                else:
                    buf = None
                    for x, g in lv:
                        buf = ops.wgrad_skinny(x, g, with_bias=True, accumulate_into=buf)
                    gw, gb = buf
            else:
                gw, gb = acc.pop("buf")
            acc["k"] = 0  # (a second backward of the same graph starts over)
        else:
            gw, gb = ops.wgrad_skinny(share, g16, with_bias=True)
        return (gx, gw[..., :A].contiguous(), gb[:A], gw[..., A:A + D].contiguous(), gb[A:A + D],
                None, None, None, None)


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
        self.anchor_matcher = Matcher(r.IOU_THRESHOLDS, r.IOU_LABELS, allow_low_quality_matches=True)
        with arg_scope([Conv2D], weights_initializer=init.random_normal(0.01)):
            self.rpn_head = build_rpn_head(cfg, shapes, scope="rpn_head")

    def _all_anchors(self, feats):
        """Level-major concatenation of the grid anchors (box_list_ops.concatenate
        of anchor_generator(features), rpn_outputs.py:253), cached per grid."""
        key = tuple((f.shape[1], f.shape[2]) for f in feats) + (str(feats[0].device),)
        if getattr(self, "_anchor_key", None) != key:
            grids = [(f.shape[1], f.shape[2]) for f in feats]
            self._anchors = torch.cat(self.anchor_generator.grid_anchors(grids, feats[0].device))
            self._anchor_key = key
        return self._anchors

    def losses(self, images, feats, logits, deltas, gt):
        """RPNOutputs.losses (rpn_outputs.py:306-401): IoU(GT, all anchors),
        Matcher(0.3/0.7, low-quality), subsample 256 @ 0.5, sigmoid CE + smooth-L1,
        both summed and normalised by BATCH_SIZE_PER_IMAGE * N."""
        anchors = self._all_anchors(feats)
        N = logits[0].shape[0]
        gt_boxes = gt["gt_boxes"]
        valid = gt["is_valid"]
        crowd = gt.get("gt_is_crowd")
        crowd = crowd.bool() if crowd is not None else torch.zeros_like(valid)
        matches, labels = match_boxes(self.anchor_matcher, gt_boxes, valid, anchors,
                                      crowd=crowd)
        if self.boundary_threshold >= 0:
            # legacy inside_window filter (rpn_outputs.py:268-277, box_list_ops.py:150)
            t = float(self.boundary_threshold)
            hw = images.image_shapes.to(anchors.dtype)
            inside = ((anchors[None, :, 0] >= -t) & (anchors[None, :, 1] >= -t) &
                      (anchors[None, :, 2] <= hw[:, :1] + t) & (anchors[None, :, 3] <= hw[:, 1:2] + t))
            labels = torch.where(inside, labels, torch.full_like(labels, -1))
        pos, neg = subsample_labels(labels, self.batch_size_per_image, self.positive_fraction, 0)
        norm = 1.0 / (self.batch_size_per_image * N)
        concat = getattr(logits, "concat", None)
        if concat is not None:  # the fused head's outputs are already in this layout
            pl, pd = concat
        else:
            pl = torch.cat([x.reshape(N, -1) for x in logits], dim=1)
            pd = torch.cat([x.reshape(N, -1, 4) for x in deltas], dim=1)
        if pl.is_cuda and gt_boxes.shape[1] > 0:
            # one HIP pass each way: targets, sigmoid CE and smooth-L1 fused
            # the normaliser x loss weight folded into the op (no multiply
            # launches either way)
            loss_cls, loss_loc = ops.rpn_loss(pl, pd, anchors, gt_boxes, matches, pos, pos | neg,
                                              self.box2box_transform.weights,
                                              self.smooth_l1_beta,
                                              scale=norm * self.loss_weight)
            return {"loss_rpn_cls": loss_cls, "loss_rpn_loc": loss_loc}
        matched = torch.gather(gt_boxes, 1, matches[..., None].expand(-1, -1, 4))
        gt_deltas = self.box2box_transform.get_deltas(
            anchors[None].expand(N, -1, -1).reshape(-1, 4), matched.reshape(-1, 4)).reshape(N, -1, 4)
        # only positive rows carry targets (dynamic_stitch of zeros, rpn_outputs.py:286-290);
        # other rows may be matched to padded GT whose log-size is -inf
        gt_deltas = torch.where(pos[..., None], gt_deltas, torch.zeros_like(gt_deltas))
        sampled = pos | neg
        obj = torch.nn.functional.binary_cross_entropy_with_logits(
            pl, pos.to(pl.dtype), reduction="none")
        loss_cls = torch.where(sampled, obj, torch.zeros_like(obj)).sum()
        loc = smooth_l1_loss(labels=gt_deltas, predictions=pd, beta=self.smooth_l1_beta)
        loss_loc = torch.where(pos[..., None], loc, torch.zeros_like(loc)).sum()
        return {"loss_rpn_cls": loss_cls * norm * self.loss_weight,
                "loss_rpn_loc": loss_loc * norm * self.loss_weight}

    def call(self, images, features, gt_instances=None):
        feats = [features[f] for f in self.in_features]
        rpn_features, logits, deltas = self.rpn_head(feats)
        losses = {}
        if self.training:
            if gt_instances is None:
                raise ValueError("RPN training needs gt_instances")
            losses = self.losses(images, feats, logits, deltas, gt_instances)
            logits = [x.detach() for x in logits]
            deltas = [x.detach() for x in deltas]
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
