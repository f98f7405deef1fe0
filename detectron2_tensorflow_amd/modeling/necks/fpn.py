"""FPN neck (lib/modeling/necks/fpn.py:31-217) on the MFMA conv kernel.

Top-down pass (fpn.py:138-149): the lateral 1x1 conv of level i runs with the
nearest-x2 upsample of the previous merged map added in its epilogue, so
``prev = lateral(x) + up2(prev)`` is one kernel (no upsampled copy, no extra
read/write of the merged map).  Output convs are 3x3 implicit GEMM on MFMA.
LastLevelMaxPool is max_pool k1/s2 = p5[:, ::2, ::2] (fpn.py:171-183);
LastLevelP6P7 returns post-ReLU p6 and p7 = conv3x3/2(p6) (fpn.py:186-217).
"""
import math
import os

import torch

from ...layers import Conv2D, Layer, ShapeSpec, get_norm, subsample, upsample
from ...layers import initializers as init
from ...utils.arg_scope import arg_scope
from .build import NECK_REGISTRY


def assert_strides_are_log2_contiguous(strides):
    for i, stride in enumerate(strides[1:], 1):
        assert stride == strides[i - 1] * 2, f"Strides {stride} {strides[i - 1]} are not log2 contiguous"


class LastLevelMaxPool(Layer):
    num_levels = 1
    in_feature = "p5"

    def call(self, x):
        return [subsample(x, 2)]


class LastLevelP6P7(Layer):
    num_levels = 2
    in_feature = "res5"

    def __init__(self, in_channels, out_channels, **kwargs):
        super().__init__(**kwargs)
        with arg_scope([Conv2D], kernel_size=3, stride=2, padding="SAME",
                       weights_initializer=init.variance_scaling(1.0)):
            self.p6 = Conv2D(in_channels, out_channels, activation="relu", scope="p6")
            self.p7 = Conv2D(out_channels, out_channels, scope="p7")

    def call(self, c5):
        p6 = self.p6(c5)
        return [p6, self.p7(p6)]


@NECK_REGISTRY.register()
class FPN(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        self.in_features = list(cfg.MODEL.NECK.IN_FEATURES)
        self.in_strides = [input_shape[f].stride for f in self.in_features]
        self.in_channels = [input_shape[f].channels for f in self.in_features]
        assert_strides_are_log2_contiguous(self.in_strides)
        self.out_channels = cfg.MODEL.NECK.OUT_CHANNELS
        self.norm = cfg.MODEL.NECK.NORM
        self.top_block_type = cfg.MODEL.NECK.TOP_BLOCK_TYPE
        self.fuse_type = cfg.MODEL.NECK.FUSE_TYPE
        assert self.fuse_type in ("avg", "sum"), self.fuse_type
        use_bias = self.norm == ""
        normalizer = get_norm(self.norm)
        lateral, output = [], []
        with arg_scope([Conv2D], use_bias=use_bias, normalizer=normalizer,
                       normalizer_params={"scope": "norm"},
                       weights_initializer=init.variance_scaling(1.0)):
            for idx, cin in enumerate(self.in_channels):
                stage = int(math.log2(self.in_strides[idx]))
                lateral.append(Conv2D(cin, self.out_channels, 1, use_bias=use_bias,
                                      normalizer=normalizer, scope=f"fpn_lateral{stage}"))
                output.append(Conv2D(self.out_channels, self.out_channels, 3, stride=1,
                                     normalizer=normalizer, scope=f"fpn_output{stage}"))
        # top-down order (low -> high resolution)
        self.lateral_convs = torch.nn.ModuleList(lateral[::-1])
        self.output_convs = torch.nn.ModuleList(output[::-1])
        if self.top_block_type == "MAXPOOL":
            self.top_block = LastLevelMaxPool(scope="top_block")
        elif self.top_block_type == "P6P7":
            cin = self.in_channels[self.in_features.index(LastLevelP6P7.in_feature)]
            self.top_block = LastLevelP6P7(cin, self.out_channels, scope="top_block")
        else:
            self.top_block = None
        self._out_feature_strides = {f"p{int(math.log2(s))}": s for s in self.in_strides}
        stage = int(math.log2(self.in_strides[-1]))
        if self.top_block is not None:
            for s in range(stage, stage + self.top_block.num_levels):
                self._out_feature_strides[f"p{s + 1}"] = 2 ** (s + 1)
        self._out_features = sorted(self._out_feature_strides)
        self._out_feature_channels = {k: self.out_channels for k in self._out_features}
        self._size_divisibility = self.in_strides[-1]

    @property
    def size_divisibility(self):
        return self._size_divisibility

    # A bottom-up feature that is also the input of the next ResNet stage (its
    # conv1 / projection-shortcut pair) and read by nothing else: the lateral
    # joins that pair's gradient hand-off, so the last of the three backwards
    # forms the feature's whole gradient with its ReLU mask (no autograd add,
    # no threshold pass; layers/convolutional.py:_join_backward).
    JOIN_GRAD = os.environ.get("D2MI_FPN_JOIN", "1") != "0"

    def _join_of(self, name, feats):
        if not self.JOIN_GRAD:
            return None
        if self.top_block is not None and getattr(self.top_block, "in_feature", None) == name:
            return None  # a third reader (P6 from C5)
        return getattr(feats, "_d2mi_pair", None)

    # A merged map read by its output conv and, as the top-down input, by the
    # next finer lateral: the two backwards hand its gradient over (the second
    # adds it; the output conv inside its dgrad epilogue) instead of an
    # autograd add of two full maps (layers/convolutional.py ctx.td_pair).
    TD_HANDOFF = os.environ.get("D2MI_FPN_TD", "1") != "0"

    def _out(self, out, prev, fused):
        if not (fused and self.TD_HANDOFF and torch.is_grad_enabled() and prev.requires_grad):
            return out(prev)
        td = {"td": True}
        y = out(prev, pair_grad=td)
        prev._d2mi_td_pair = td  # (read by the finer lateral's forward)
        return y

    def call(self, bottom_up_features):
        names = self.in_features[::-1]
        x = [bottom_up_features[f] for f in names]
        fused = self.fuse_type == "sum" and self.norm == ""
        prev = self.lateral_convs[0](x[0], join=self._join_of(names[0], x[0]))
        results = [self._out(self.output_convs[0], prev, fused)]
        for name, feats, lat, out in zip(names[1:], x[1:], self.lateral_convs[1:],
                                         self.output_convs[1:]):
            if fused:
                # lateral + up2(prev) in one kernel
                prev = lat(feats, topdown=prev, join=self._join_of(name, feats))
            else:
                prev = lat(feats) + upsample(prev, 2)
                if self.fuse_type == "avg":
                    prev = prev / 2
            results.insert(0, self._out(out, prev, fused))
        if self.top_block is not None:
            src = bottom_up_features.get(self.top_block.in_feature)
            if src is None:
                src = results[self._out_features.index(self.top_block.in_feature)]
            results.extend(self.top_block(src))
        assert len(self._out_features) == len(results)
        return dict(zip(self._out_features, results))

    def output_shape(self):
        return {n: ShapeSpec(channels=self._out_feature_channels[n], stride=self._out_feature_strides[n])
                for n in self._out_features}
