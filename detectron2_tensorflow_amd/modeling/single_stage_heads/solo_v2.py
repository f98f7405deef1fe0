"""SOLOv2Head inference (lib/modeling/single_stage_heads/solo_v2.py:67-721).

MaskKernelBranch (:121-272): per level the FPN map (p2 resized to p3's size,
p6 to p5's, :221-239) with two coordinate channels appended (:257-263) is
resized to the S x S grid (TF bilinear, the HIP ResizeBilinear kernel),
then two towers of 4 x (3x3 conv -> GroupNorm(32) -> ReLU) run on the MFMA
conv kernel: the category tower (on the map without the coordinates) ends
in solo_cate (3x3, K classes), the kernel tower (258 input channels: zero
channels appended to 260 for the MFMA tiles) in solo_kernel (3x3, D = 256
dynamic-kernel weights per cell).

MaskFeatureBranch (:630-721): per level p2..p5 a chain of 3x3 conv -> GN ->
ReLU (-> nearest x2: the reference's Upsample(method="bilinear") ignores the
method, lib/layers/wrappers.py:104-116) down to stride 4, summed, then a
1x1 conv -> GN -> ReLU to D channels; p5 gets the coordinate channels.

Inference (:476-627) is ops.solo_inference (csrc/solo.hip): point NMS,
live cells, one dynamic 1x1 conv GEMM per image on MFMA, mask statistics,
candidate top-k, Matrix NMS, pad, masks resized to the padded image, boxes
from the masks.  Output masks are uint8 0/1 (the reference's float 0/1).

Strides: the reference's split_features multiplies strides[0] by 2 and
divides strides[-1] by 2 on EVERY call (:237-238, a bug not reproduced); the
first call's values ([8, 8, 16, 32, 32] for p2..p6) are used.
Training (:274-474): get_ground_truth as batched tensor ops (solov2_targets)
and the dice + focal losses (MaskKernelBranch.losses); the dynamic 1x1 conv
runs only for the positive cells (the reference convolves every cell's
kernel, then gathers the positives: the same products).
"""
import numpy as np
import torch

from ...layers import Conv2D, GroupNorm, Layer, Sequential, Upsample
from ...layers import initializers as init
from ...layers import ops
from ...layers.loss import dice_loss, sigmoid_focal_loss
from ...layers.functional import resize_images
from ...structures import BoxList
from ...utils.arg_scope import arg_scope
from .build import SINGLE_STAGE_HEADS_REGISTRY

_LIN_CACHE = {}


def linspace_tf(num, device):
    """tf.linspace(-1., 1., num) in float32 (TF LinSpaceOp: start + step * i,
    step = (stop - start) / (num - 1), the last value exactly stop)."""
    key = (int(num), str(device))
    v = _LIN_CACHE.get(key)
    if v is None:
        n = int(num)
        if n == 1:
            a = np.array([-1.0], np.float32)
        else:
            step = np.float32(2.0) / np.float32(n - 1)
            a = np.float32(-1.0) + step * np.arange(n, dtype=np.float32)
            a[-1] = np.float32(1.0)
        v = torch.from_numpy(a.astype(np.float32)).to(device)
        _LIN_CACHE[key] = v
    return v


def coord_channels(N, H, W, device):
    """[N, H, W, 2] = (xx, yy) of tf.meshgrid(linspace(W), linspace(H))
    (solo_v2.py:258-262, :712-716)."""
    x = linspace_tf(W, device)
    y = linspace_tf(H, device)
    xx = x.view(1, 1, W, 1).expand(N, H, W, 1)
    yy = y.view(1, H, 1, 1).expand(N, H, W, 1)
    return torch.cat([xx, yy], dim=3)


def tf_resize_bilinear(x, oh, ow):
    """TF ResizeBilinear with half-pixel centres on [P, H, W] float32 in
    torch, the TF arithmetic op for op (the oracle's resize_bilinear_tf):
    the gt-mask resample of get_ground_truth (solo_v2.py:468-471), on any
    device."""
    P, H, W = x.shape
    dev = x.device

    def interp(o, i):
        scale = torch.tensor(np.float32(i) / np.float32(o), device=dev)
        v = (torch.arange(o, device=dev, dtype=torch.float32) + 0.5) * scale - 0.5
        f = torch.floor(v)
        lo = f.to(torch.int64).clamp(min=0)
        hi = torch.ceil(v).to(torch.int64).clamp(max=i - 1)
        return lo, hi, v - f

    ylo, yhi, yl = interp(oh, H)
    xlo, xhi, xl = interp(ow, W)
    top_rows, bot_rows = x[:, ylo], x[:, yhi]
    tl, tr = top_rows[:, :, xlo], top_rows[:, :, xhi]
    bl, br = bot_rows[:, :, xlo], bot_rows[:, :, xhi]
    xl_, yl_ = xl.view(1, 1, ow), yl.view(1, oh, 1)
    top = tl + (tr - tl) * xl_
    bottom = bl + (br - bl) * xl_
    return top + (bottom - top) * yl_


def _floordiv(x, g):
    """TF FloorDiv of a float32 tensor by the Python float 1. / g (a float32
    constant): floor(x / f32(1 / g))."""
    return torch.floor(x / torch.tensor(np.float32(1.0 / g), device=x.device))


def solov2_targets(gt_boxes, gt_classes, is_valid, gt_masks, mask_hw, num_grids, scale_ranges,
                   sigma):
    """get_ground_truth (solo_v2.py:373-474) on a dense batch: gt_boxes
    [N, G, 4] yxyx image px, gt_classes [N, G], is_valid [N, G], gt_masks
    [N, G, Hi, Wi] 0/1 at the padded image size, mask_hw the mask-feature
    size.  Per level (classes [N, S, S] int64, 0 = no object; positives
    [P, 2] = (image, cell) in tf.where order: GT, then row, then column;
    target masks [P, Hm, Wm] float32).  center_of_mass is the reference's
    mean of mask x coordinate over all pixels (:43-64), from exact sums;
    a cell two GT of a level claim takes the later GT's class."""
    dev = gt_boxes.device
    N = gt_boxes.shape[0]
    vb, vg = torch.nonzero(is_valid.bool(), as_tuple=True)
    boxes = gt_boxes[vb, vg].float()
    classes = gt_classes[vb, vg].long()
    masks = gt_masks[vb, vg]
    Hi, Wi = masks.shape[1:]
    h, w = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
    area_sqrt = torch.sqrt(h * w)
    sig = torch.tensor(np.float32(sigma), device=dev)
    half_h, half_w = 0.5 * h * sig, 0.5 * w * sig
    Hm, Wm = int(mask_hw[0]), int(mask_hw[1])
    up_h = torch.tensor(np.float32(Hm * 4), device=dev)
    up_w = torch.tensor(np.float32(Wm * 4), device=dev)
    # exact coordinate sums (integers, float64), then the mean in float32
    m64 = masks.to(torch.float64)
    rows = m64.sum(2)                               # [V, Hi]
    cols = m64.sum(1)                               # [V, Wi]
    cy_all = ((rows * torch.arange(Hi, device=dev, dtype=torch.float64)).sum(1)
              / (Hi * Wi)).float()
    cx_all = ((cols * torch.arange(Wi, device=dev, dtype=torch.float64)).sum(1)
              / (Hi * Wi)).float()
    out = []
    for (lo, hi), S in zip(scale_ranges, num_grids):
        sel = torch.nonzero((area_sqrt >= np.float32(lo)) & (area_sqrt <= np.float32(hi)),
                            as_tuple=True)[0]
        ch, cw = cy_all[sel], cx_all[sel]
        coord_h = _floordiv(ch / up_h, S)
        coord_w = _floordiv(cw / up_w, S)
        zero = torch.zeros_like(ch)
        top = torch.maximum(coord_h - 1, torch.maximum(zero, _floordiv((ch - half_h[sel]) / up_h, S)))
        down = torch.minimum(coord_h + 1, torch.minimum(zero + (S - 1),
                                                        _floordiv((ch + half_h[sel]) / up_h, S)))
        left = torch.maximum(coord_w - 1, torch.maximum(zero, _floordiv((cw - half_w[sel]) / up_w, S)))
        right = torch.minimum(coord_w + 1, torch.minimum(zero + (S - 1),
                                                         _floordiv((cw + half_w[sel]) / up_w, S)))
        g = torch.arange(S, device=dev, dtype=torch.float32)
        yy, xx = g.view(1, S, 1), g.view(1, 1, S)
        pos = ((yy >= top.view(-1, 1, 1)) & (yy <= down.view(-1, 1, 1))
               & (xx >= left.view(-1, 1, 1)) & (xx <= right.view(-1, 1, 1)))
        k, py, px = torch.nonzero(pos, as_tuple=True)
        b = vb[sel][k]
        cell = py * S + px
        cls_map = torch.zeros(N * S * S, dtype=torch.int64, device=dev)
        if k.numel():
            # the later positive of a cell wins (a scatter of the ordinal, max)
            flat = b * S * S + cell
            order = torch.arange(k.numel(), device=dev)
            win = torch.full((N * S * S,), -1, dtype=torch.int64, device=dev)
            win.scatter_reduce_(0, flat, order, reduce="amax")
            hit = win >= 0
            cls_map[hit] = classes[sel][k[win[hit]]]
            tm = torch.round(tf_resize_bilinear(masks[sel].float(), Hm, Wm))[k]
        else:
            tm = torch.zeros((0, Hm, Wm), dtype=torch.float32, device=dev)
        out.append((cls_map.view(N, S, S), torch.stack([b, cell], 1), tm))
    return out


def _gn_params():
    return {"num_groups": 32, "scope": "norm"}


class MaskKernelBranch(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        s = cfg.MODEL.SOLO
        self.num_classes = cfg.MODEL.SINGLE_STAGE_HEAD.NUM_CLASSES
        self.in_features = list(cfg.MODEL.SINGLE_STAGE_HEAD.IN_FEATURES)
        strides = [float(input_shape[f].stride) for f in self.in_features]
        strides[0] *= 2
        strides[-1] /= 2
        self.strides = strides
        self.num_grids = list(s.NUM_GRIDS)
        self.scale_ranges = [tuple(r) for r in s.SCALE_RANGES]
        self.sigma = s.SIGMA
        self.focal_loss_alpha = s.FOCAL_LOSS_ALPHA
        self.focal_loss_gamma = s.FOCAL_LOSS_GAMMA
        self.ins_loss_weight = s.INS_LOSS_WEIGHT
        self.mask_kernel_size = s.MASK_KERNEL_SIZE
        self.mask_feature_out_dims = s.MASK_FEATURE_OUT_DIMS
        self.score_threshold = s.SCORE_THRESH_TEST
        self.update_score_threshold = s.UPDATE_SCORE_THRESH_TEST
        self.pre_nms_topk = s.TOPK_CANDIDATES_TEST
        self.mask_threshold = s.MASK_THRESH_TEST
        self.nms_kernel = s.NMS_KERNEL
        self.nms_sigma = s.NMS_SIGMA
        self.max_detections_per_image = cfg.TEST.DETECTIONS_PER_IMAGE
        if s.USE_DEFORM_CONV:
            raise NotImplementedError("deformable convs are outside the hot path (SURVEY section 2)")
        if self.mask_kernel_size != 1:
            raise NotImplementedError("MASK_KERNEL_SIZE > 1 (a KxK dynamic conv) is not shipped "
                                      "by any reference config")
        cin = input_shape[self.in_features[0]].channels
        dims = s.MASK_KERNEL_CONVS_DIM
        kernel_dims = self.mask_feature_out_dims * self.mask_kernel_size ** 2
        norm = GroupNorm if s.MASK_KERNEL_NORM == "GN" else None
        prior = s.PRIOR_PROB
        with arg_scope([Conv2D], kernel_size=3, stride=1, padding="SAME", use_bias=norm is None,
                       normalizer=norm, normalizer_params=_gn_params() if norm else None,
                       activation="relu", weights_initializer=init.random_normal(0.01)):
            cls, ker = [], []
            for i in range(s.MASK_KERNEL_NUM_CONVS):
                cls.append(Conv2D(cin if i == 0 else dims, dims, scope=f"cate_subnet{2 * i}"))
                ker.append(Conv2D(cin + 2 if i == 0 else dims, dims, scope=f"kernel_subnet{2 * i}"))
            self.cls_layers = torch.nn.ModuleList(cls)
            self.kernel_layers = torch.nn.ModuleList(ker)
            self.cls_subnet = Sequential(cls)
            self.kernel_subnet = Sequential(ker)
            self.solo_cate = Conv2D(dims, self.num_classes, activation=None, use_bias=True,
                                    normalizer=None,
                                    bias_initializer=init.constant(-np.log((1 - prior) / prior)),
                                    scope="solo_cate")
            self.solo_kernel = Conv2D(dims, kernel_dims, activation=None, use_bias=True,
                                      normalizer=None, scope="solo_kernel")

    def split_features(self, features):
        f = [features[k] for k in self.in_features]
        p3_hw = f[1].shape[1:3]
        p5_hw = f[3].shape[1:3]
        return [resize_images(f[0], p3_hw), f[1], f[2], f[3], resize_images(f[4], p5_hw)]

    def grid_inputs(self, features):
        """Per level (cls-tower input [N,S,S,C], kernel-tower input [N,S,S,C+2]).
        The resize is per channel, so resizing the map and the coordinate
        channels separately equals resizing their concatenation."""
        out = []
        for i, f in enumerate(self.split_features(features)):
            N, H, W, _ = f.shape
            S = self.num_grids[i]
            g = resize_images(f, (S, S))
            gc = resize_images(coord_channels(N, H, W, f.device).contiguous(), (S, S))
            out.append((g, torch.cat([g, gc], dim=3)))
        return out

    def call(self, features):
        """(category logits [N,S,S,K] per level, kernels [N,S,S,D] per level);
        the sigmoid + point NMS of the inference path run in ops.solo_inference."""
        ins = self.grid_inputs(features)
        c = [g for g, _ in ins]
        k = [gk for _, gk in ins]
        # each tower layer over all five grids in one multi-level launch
        for layer in self.cls_layers:
            c = layer.call_levels(c)
        for layer in self.kernel_layers:
            k = layer.call_levels(k)
        return self.solo_cate.call_levels(c), self.solo_kernel.call_levels(k)

    def losses(self, pred_classes, pred_kernels, mask_feats, targets):
        """MaskKernelBranch.losses (solo_v2.py:274-371): dice ("mean") x
        INS_LOSS_WEIGHT over the positive cells' dynamic-conv masks, focal
        ("sum") over every cell against one_hot(class, K + 1)[:, 1:] -- the
        reference's class 0 is "no object" here (so a 0-based label L trains
        category channel L - 1, as the reference computes it) -- divided by
        (positives + 1)."""
        N, Hm, Wm, E = mask_feats.shape
        tg = solov2_targets(targets["gt_boxes"], targets["gt_classes"], targets["is_valid"],
                            targets["gt_masks"], (Hm, Wm), self.num_grids, self.scale_ranges,
                            self.sigma)
        feats = mask_feats.reshape(N, Hm * Wm, E)
        kern, pos, gts, offset = [], [], [], 0
        for (cls_map, p, tm), pk in zip(tg, pred_kernels):
            S = cls_map.shape[1]
            kern.append(pk.reshape(N, S * S, E))
            pos.append(torch.stack([p[:, 0], p[:, 1] + offset], 1))
            gts.append(tm)
            offset += S * S
        kern = torch.cat(kern, 1)
        pos = torch.cat(pos, 0)
        gts = torch.cat(gts, 0)
        masks = mask_feats.new_zeros((pos.shape[0], Hm * Wm))
        for b in range(N):  # one GEMM per image: its positive cells' kernels x its features
            rows = torch.nonzero(pos[:, 0] == b, as_tuple=True)[0]
            if rows.numel():
                masks = masks.index_copy(0, rows, kern[b, pos[rows, 1]] @ feats[b].t())
        loss_ins = dice_loss(predictions=torch.sigmoid(masks), targets=gts.reshape(-1, Hm * Wm),
                             reduction="mean") * self.ins_loss_weight
        K = self.num_classes
        logits = torch.cat([pc.reshape(-1, K) for pc in pred_classes], 0)
        labels = torch.cat([c.reshape(-1) for c, _, _ in tg], 0)
        onehot = torch.nn.functional.one_hot(labels, K + 1)[:, 1:].to(logits.dtype)
        loss_cls = sigmoid_focal_loss(predictions=logits, targets=onehot,
                                      alpha=self.focal_loss_alpha, gamma=self.focal_loss_gamma,
                                      reduction="sum")
        return {"loss_ins": loss_ins, "loss_cls": loss_cls / (pos.shape[0] + 1)}


class MaskFeatureBranch(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        s = cfg.MODEL.SOLO
        self.in_features = list(s.MASK_FEATURE_IN_FEATURES)
        strides = {k: v.stride for k, v in input_shape.items()}
        chans = {k: v.channels for k, v in input_shape.items()}
        dims = s.MASK_FEATURE_CONVS_DIM
        out_dims = s.MASK_FEATURE_OUT_DIMS
        self.common_stride = s.MASK_FEATURE_COMMON_STRIDE
        norm = GroupNorm if s.MASK_FEATURE_NORM == "GN" else None
        heads, layers = [], []
        with arg_scope([Conv2D], kernel_size=3, stride=1, padding="SAME", use_bias=norm is None,
                       normalizer=norm, normalizer_params=_gn_params() if norm else None,
                       activation="relu", weights_initializer=init.random_normal(0.01)):
            for f in self.in_features:
                head = Sequential()
                n = max(1, int(np.log2(strides[f]) - np.log2(self.common_stride)))
                cin = chans[f] + (2 if f == self.in_features[-1] else 0)
                for k in range(n):
                    conv = Conv2D(cin if k == 0 else dims, dims, scope=f"{f}_{2 * k}")
                    layers.append(conv)
                    head.add(conv)
                    if strides[f] != self.common_stride:
                        head.add(Upsample(factor=2, method="bilinear"))
                heads.append(head)
            self.scale_layers = torch.nn.ModuleList(layers)
            self.scale_heads = heads
            self.predictor = Conv2D(dims, out_dims, kernel_size=1, stride=1, padding="VALID",
                                    normalizer_params={"num_groups": 32, "scope": "norm"},
                                    scope="predictor")

    def call(self, features):
        """res = sum of the scale heads (solo_v2.py:705-721).  On the GPU in
        inference every head's last GroupNorm writes its ReLU'd, upsampled
        output straight into the running sum (d2mi_group_norm_nhwc up2 +
        accumulate): no upsampled copy, no separate add."""
        res = None
        for i, f in enumerate(self.in_features):
            x = features[f]
            if i > 0 and f == self.in_features[-1]:
                N, H, W, _ = x.shape
                x = torch.cat([x, coord_channels(N, H, W, x.device)], dim=3)
            layers = self.scale_heads[i]._layers
            convs = [m for m in layers if isinstance(m, Conv2D)]
            up = any(isinstance(m, Upsample) for m in layers)
            last = convs[-1]
            norm = last.normalizer_fn
            fusable = (res is not None and isinstance(norm, GroupNorm) and norm.fused_ok(x)
                       and last.act_fn is not None)
            if not fusable:
                y = self.scale_heads[i](x)
                res = y if res is None else res + y
                continue
            for conv in convs[:-1]:  # conv -> GN + ReLU (-> up2) chain before the last
                x = conv(x)
                if up:
                    x = x.repeat_interleave(2, 1).repeat_interleave(2, 2)
            y = last(x, raw=True)
            norm(y, relu=True, up2=up, accumulate_into=res)
        return self.predictor(res)


@SINGLE_STAGE_HEADS_REGISTRY.register()
class SOLOv2Head(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        self.mask_kernel_branch = MaskKernelBranch(cfg, input_shape, scope="mask_kernel")
        self.mask_feature_branch = MaskFeatureBranch(cfg, input_shape, scope="mask_feature")

    def call(self, images, features, targets=None):
        pred_cls, pred_kernels = self.mask_kernel_branch(features)
        mask_feats = self.mask_feature_branch(features)
        if self.training:
            if targets is None:
                raise ValueError("SOLOv2 training needs targets")
            return None, self.mask_kernel_branch.losses(pred_cls, pred_kernels, mask_feats,
                                                        targets)
        image_hw = images.tensor.shape[1:3]
        return self.inference(pred_cls, pred_kernels, mask_feats, image_hw), {}

    def inference(self, pred_cls, pred_kernels, mask_feats, image_hw, debug=None):
        b = self.mask_kernel_branch
        masks, boxes, scores, classes, valid = ops.solo_inference(
            pred_cls, pred_kernels, mask_feats, b.strides, image_hw, b.score_threshold,
            b.mask_threshold, b.update_score_threshold, b.pre_nms_topk,
            b.max_detections_per_image, b.nms_kernel, b.nms_sigma, debug=debug)
        res = BoxList(boxes)
        res.add_field("pred_classes", classes)
        res.add_field("scores", scores)
        res.add_field("is_valid", valid)
        res.add_field("pred_masks", masks)
        return res
