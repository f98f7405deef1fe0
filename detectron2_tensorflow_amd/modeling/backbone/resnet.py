"""ResNet backbone (lib/modeling/backbone/resnet.py:22-253, blocks.py:143-186).

A caller of the hot path: the bottleneck 1x1
and 3x3 convs run on the MFMA conv kernel with FrozenBN folded into the
weights at run time; the frozen stem's 7x7 (Cin = 3) runs on its own
split-bf16 MFMA kernel (d2mi_stem_conv, since r3).
Structure, strides (STRIDE_IN_1X1), the stem's zero pad + 3x3/2 VALID max
pool and FREEZE_AT follow the reference.
"""
import copy
from contextlib import ExitStack, contextmanager

import torch
import torch.nn.functional as F

from ...layers import BatchNorm, Conv2D, Layer, get_norm, ops
from ...layers.activation import is_relu
from ...layers import initializers as init
from ...utils.arg_scope import add_arg_scope, arg_scope
from .build import BACKBONE_REGISTRY, Backbone


@contextmanager
def resnet_arg_scope(freeze, norm):
    normalizer = get_norm(norm)
    with arg_scope([Conv2D], use_bias=False, normalizer=normalizer,
                   normalizer_params={"scope": "norm"}, activation="relu", impl="torch",
                   weights_initializer=init.variance_scaling(2.0, mode="fan_out")), ExitStack() as st:
        if freeze:
            st.enter_context(arg_scope([Conv2D, BatchNorm], trainable=False))
        yield


@add_arg_scope
class BottleneckBlock(Layer):
    def __init__(self, in_channels, out_channels, bottleneck_channels, stride=1, num_groups=1,
                 stride_in_1x1=False, rate=1, **kwargs):
        super().__init__(in_channels=in_channels, out_channels=out_channels, **kwargs)
        # every conv runs on the MFMA implicit-GEMM kernel with FrozenBN folded
        # and ReLU / residual fused in its epilogue ("auto": a grouped or
        # dilated 3x3 falls back to MIOpen)
        # set by Stage for blocks after the first: their input is the previous
        # block's output and nothing else reads it (see call)
        self.grad_handoff = False
        self.grad_pair = True  # conv1 / projection-shortcut pair hand-off (see call)
        self.shortcut = None
        if in_channels != out_channels:
            self.shortcut = Conv2D(in_channels, out_channels, 1, stride=stride, activation=None,
                                   impl="mfma", scope="shortcut")
        s1, s3 = (stride, 1) if stride_in_1x1 else (1, stride)
        self.conv1 = Conv2D(in_channels, bottleneck_channels, 1, stride=s1, impl="mfma",
                            scope="conv1")
        self.conv2 = Conv2D(bottleneck_channels, bottleneck_channels, 3, stride=s3,
                            num_groups=num_groups, rate=rate, impl="auto", scope="conv2")
        self.conv3 = Conv2D(bottleneck_channels, out_channels, 1, activation=None, impl="mfma",
                            scope="conv3")

    def call(self, x):
        # projection shortcut: it and conv1 both read x; their input gradients
        # meet in the second one's epilogue instead of an autograd add
        pair = ({} if self.grad_pair and self.shortcut is not None and torch.is_grad_enabled()
                else None)
        if pair is not None:
            # a later reader of x (the FPN lateral) may join the pair: see
            # layers/convolutional.py:_join_backward
            x._d2mi_pair = pair
        sc = self.shortcut(x, pair_grad=pair) if self.shortcut is not None else x
        # relu(conv3(...) + shortcut) in one kernel.  conv1 -> conv2 -> conv3 is
        # a chain of sole consumers: each one's dgrad applies the previous
        # ReLU's mask (no separate ReLU-backward pass).  With an identity
        # shortcut, conv3 hands its residual gradient to conv1, whose dgrad adds
        # it before applying the mask of x (the previous block's ReLU output,
        # read by nothing else inside a stage): conv1 then carries x's whole
        # gradient -- no autograd add, no separate ReLU backward.
        link = ({} if self.grad_handoff and self.shortcut is None and torch.is_grad_enabled()
                else None)
        h = self.conv1(x, relu_input_sole_consumer=link is not None, grad_from=link, pair_grad=pair)
        h = self.conv2(h, relu_input_sole_consumer=True)
        return self.conv3(h, residual=sc.contiguous(), final_relu=True,
                          relu_input_sole_consumer=True, res_grad_to=link)


@add_arg_scope
class Stem(Layer):
    def __init__(self, in_channels, out_channels, **kwargs):
        super().__init__(in_channels=in_channels, out_channels=out_channels, **kwargs)
        self.conv1 = Conv2D(in_channels, out_channels, 7, stride=2,
                            normalizer_params={"channels": out_channels, "scope": "norm"},
                            scope="conv1")

    def _fused_ok(self, x):
        c = self.conv1
        needs_grad = torch.is_grad_enabled() and (x.requires_grad or c.fold_trainable())
        return (x.is_cuda and not needs_grad and is_relu(c.act_fn) and c.padding == "SAME"
                and c.rate == 1 and c.num_groups == 1 and c.out_channels % 4 == 0)

    # the frozen stem's conv on the split-bf16 MFMA stem kernel (d2mi_stem_conv;
    # False: MIOpen, the A/B arm)
    MFMA_CONV = True

    def call(self, x):
        if self._fused_ok(x):
            # frozen stem: the 7x7 conv without its bias, then relu(+ shift),
            # the zero pad and the 3x3/2 pool in one HIP pass (ops.stem_pool)
            c = self.conv1
            w, b, norm, _ = c.effective_params()
            if norm is None:
                if (self.MFMA_CONV and tuple(w.shape) == (7, 7, 3, 64) and c.stride == 2
                        and x.shape[-1] == 3):
                    key = c._param_key()  # (the fold is cached on the same versions)
                    if getattr(self, "_w3_key", None) != key:
                        self._w3 = ops.stem_conv_weights(w)
                        self._w3_key = key
                    return ops.stem_pool(ops.stem_conv(x, self._w3), b)
                p = (c.kernel_size - 1) // 2
                y = F.conv2d(x.permute(0, 3, 1, 2),
                             w.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last),
                             None, stride=c.stride, padding=p)
                return ops.stem_pool(y.permute(0, 2, 3, 1), b)
        ret = self.conv1(x)
        ret = F.pad(ret.permute(0, 3, 1, 2), (1, 1, 1, 1))  # tf.pad zeros (resnet.py:80)
        ret = F.max_pool2d(ret, 3, 2)                        # VALID 3x3/2 (resnet.py:81)
        return ret.permute(0, 2, 3, 1)

    @property
    def stride(self):
        return 4


class Stage(Layer):
    def __init__(self, block_class, block_kwargs, num_blocks, first_stride, **kwargs):
        super().__init__(**kwargs)
        self.blocks = torch.nn.ModuleList()
        for i in range(num_blocks):
            kw = copy.copy(block_kwargs)
            kw["scope"] = f"block_{i + 1}"
            kw["stride"] = first_stride if i == 0 else 1
            if i > 0:
                kw["in_channels"] = block_kwargs["out_channels"]
            self.blocks.append(block_class(**kw))
            if i > 0 and hasattr(self.blocks[-1], "grad_handoff"):
                self.blocks[-1].grad_handoff = True

    def call(self, x):
        for b in self.blocks:
            x = b(x)
        return x


@BACKBONE_REGISTRY.register()
class ResNet(Backbone):
    def __init__(self, cfg, input_shape, **kwargs):
        r = cfg.MODEL.RESNETS
        if r.RES5_DILATION not in (1, 2):
            raise ValueError(f"res5_dilation cannot be {r.RES5_DILATION}.")
        if any(r.DEFORM_ON_PER_STAGE):
            raise NotImplementedError("deformable ResNet stages are outside the hot path")
        super().__init__(**kwargs)
        self._out_features = list(r.OUT_FEATURES)
        freeze_at = cfg.MODEL.BACKBONE.FREEZE_AT
        out_stage_idx = [{"res2": 2, "res3": 3, "res4": 4, "res5": 5}[f] for f in self._out_features]
        max_stage_idx = max(out_stage_idx)
        num_blocks = {50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}[r.DEPTH]
        with resnet_arg_scope(freeze_at > 0, r.NORM):
            self.stem = Stem(input_shape.channels, r.STEM_OUT_CHANNELS, scope="stem")
        stride = self.stem.stride
        self._out_feature_strides = {"stem": stride}
        self._out_feature_channels = {"stem": r.STEM_OUT_CHANNELS}
        in_ch, out_ch = r.STEM_OUT_CHANNELS, r.RES2_OUT_CHANNELS
        bott = r.NUM_GROUPS * r.WIDTH_PER_GROUP
        self.stages = torch.nn.ModuleList()
        self.stage_names = []
        for idx, stage_idx in enumerate(range(2, max_stage_idx + 1)):
            rate = r.RES5_DILATION if stage_idx == 5 else 1
            first_stride = 1 if (idx == 0 or (stage_idx == 5 and rate == 2)) else 2
            kw = {"in_channels": in_ch, "out_channels": out_ch, "bottleneck_channels": bott,
                  "rate": rate, "num_groups": r.NUM_GROUPS, "stride_in_1x1": r.STRIDE_IN_1X1}
            name = f"res{stage_idx}"
            with resnet_arg_scope(freeze_at >= stage_idx, r.NORM):
                self.stages.append(Stage(BottleneckBlock, kw, num_blocks[idx], first_stride,
                                         scope=name))
            self.stage_names.append(name)
            stride = int(stride * first_stride)
            self._out_feature_strides[name] = stride
            self._out_feature_channels[name] = out_ch
            in_ch, out_ch, bott = out_ch, out_ch * 2, bott * 2

    def call(self, x):
        outputs = {}
        x = self.stem(x)
        if "stem" in self._out_features:
            outputs["stem"] = x
        for name, stage in zip(self.stage_names, self.stages):
            x = stage(x)
            if name in self._out_features:
                outputs[name] = x
        return outputs
