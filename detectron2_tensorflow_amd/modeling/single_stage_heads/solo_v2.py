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
Training (dice + focal losses, :274-474) is outside the hot path: raises.
"""
import numpy as np
import torch

from ...layers import Conv2D, GroupNorm, Layer, Sequential, Upsample
from ...layers import initializers as init
from ...layers import ops
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
        if self.training:
            raise NotImplementedError("SOLOv2 training (dice + focal losses) is outside the hot "
                                      "path: BASELINE config C5 is the inference tail")
        image_hw = images.tensor.shape[1:3]
        pred_cls, pred_kernels = self.mask_kernel_branch(features)
        mask_feats = self.mask_feature_branch(features)
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
