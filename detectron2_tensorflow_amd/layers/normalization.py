"""BatchNorm / GroupNorm / get_norm (lib/layers/normalization.py:15-274).

The hot-path configs use FrozenBN in the backbone (MODEL.RESNETS.NORM) and no
norm in FPN / heads.  BatchNorm here implements the inference form (moving
statistics, which is what FrozenBN and training=False use):
    y = x * gamma * rsqrt(var + eps) + (beta - mean * gamma * rsqrt(var + eps)).
Training-mode batch statistics and SyncBN (broken in the reference,
normalization.py:121-168) are not part of the hot path.
"""
import torch

from ..utils.arg_scope import add_arg_scope
from . import ops
from .base import Layer


@add_arg_scope
class BatchNorm(Layer):
    def __init__(self, channels, momentum=0.997, epsilon=1e-5, center=True, scale=True,
                 trainable=True, sync=False, **kwargs):
        kwargs.pop("training", None)
        super().__init__(channels=channels, momentum=momentum, epsilon=epsilon, center=center,
                         scale_=scale, trainable=trainable, sync=sync, training=False, **kwargs)
        self.beta = torch.nn.Parameter(torch.zeros(channels), requires_grad=trainable) if center else None
        self.gamma = torch.nn.Parameter(torch.ones(channels), requires_grad=trainable) if scale else None
        self.register_buffer("moving_mean", torch.zeros(channels))
        self.register_buffer("moving_variance", torch.ones(channels))

    def folded(self):
        """(scale, shift) of the frozen affine transform."""
        inv = torch.rsqrt(self.moving_variance + self.epsilon)
        scale = inv * self.gamma if self.gamma is not None else inv
        shift = -self.moving_mean * scale
        if self.beta is not None:
            shift = shift + self.beta
        return scale, shift

    def call(self, x):
        scale, shift = self.folded()
        return x * scale + shift


@add_arg_scope
class GroupNorm(Layer):
    def __init__(self, channels, num_groups=32, epsilon=1e-5, trainable=True, **kwargs):
        super().__init__(channels=channels, num_groups=num_groups, epsilon=epsilon, **kwargs)
        self.gamma = torch.nn.Parameter(torch.ones(channels), requires_grad=trainable)
        self.beta = torch.nn.Parameter(torch.zeros(channels), requires_grad=trainable)

    def fused_ok(self, x):
        """The HIP GroupNorm (d2mi_group_norm_nhwc, no autograd) takes the call
        only when no gradient is needed at all: neither the input nor the
        affine parameters require one (a frozen GN in a trainable branch must
        still pass the input gradient through torch's group_norm)."""
        C = self.channels
        needs_grad = torch.is_grad_enabled() and (
            x.requires_grad or self.gamma.requires_grad or self.beta.requires_grad)
        return (x.is_cuda and not needs_grad
                and C % self.num_groups == 0 and (C // self.num_groups) % 4 == 0 and C <= 1024
                and self.num_groups <= 64)

    def call(self, x, relu=False, up2=False, accumulate_into=None):
        """GroupNorm.call (normalization.py:235-260) on NHWC.  relu / up2 /
        accumulate_into fuse the ops that follow it in the SOLOv2 heads (HIP
        path); training (autograd) runs on torch's group_norm."""
        if self.fused_ok(x):
            return ops.group_norm(x, self.num_groups, self.gamma, self.beta, self.epsilon,
                                  relu, up2, accumulate_into)
        y = torch.nn.functional.group_norm(x.permute(0, 3, 1, 2), self.num_groups, self.gamma,
                                           self.beta, self.epsilon).permute(0, 2, 3, 1)
        if relu:
            y = torch.relu(y)
        if up2:
            y = y.repeat_interleave(2, 1).repeat_interleave(2, 2)
        if accumulate_into is not None:
            return accumulate_into.add_(y)
        return y


def get_norm(norm):
    if isinstance(norm, str):
        if len(norm) == 0:
            return None
        if norm == "GN":
            return GroupNorm
        if norm in ("BN", "FrozenBN", "SyncBN"):
            return BatchNorm
        raise ValueError(f"{norm} is not recognized !")
    return norm
