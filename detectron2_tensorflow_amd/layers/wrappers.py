"""Linear / Upsample / MaxPool2D (lib/layers/wrappers.py:13-131)."""
import torch
import torch.nn.functional as F

from ..utils.arg_scope import add_arg_scope
from . import initializers as init
from .activation import get_activation
from .base import Layer
from .convolutional import fix_padding
from .functional import upsample


@add_arg_scope
class Linear(Layer):
    """x @ weights + bias with weights [in_units, out_units] (TF Dense layout);
    the GEMM is a plain library GEMM (hipBLASLt through torch.addmm)."""

    def __init__(self, in_units, out_units, activation=None, normalizer=None,
                 normalizer_params=None, use_bias=True, weights_initializer=None,
                 weights_regularizer=None, bias_initializer=None, bias_regularizer=None,
                 variables_collections=None, trainable=True, outputs_collections=None, **kwargs):
        super().__init__(in_units=int(in_units), out_units=int(out_units), activation=activation,
                         use_bias=use_bias, trainable=trainable, **kwargs)
        w = torch.empty((int(in_units), int(out_units)))
        (weights_initializer or init.variance_scaling(1.0, mode="fan_avg", distribution="uniform"))(w)
        self.weights = torch.nn.Parameter(w, requires_grad=trainable)
        self.bias = torch.nn.Parameter(torch.zeros(int(out_units)), requires_grad=trainable) if use_bias else None
        self.normalizer_fn = None
        if normalizer is not None:
            self.normalizer_fn = normalizer(**(normalizer_params or {}))
        self.act_fn = get_activation(activation)

    def call(self, inputs):
        x = inputs.reshape(inputs.shape[0], -1) if inputs.dim() > 2 else inputs
        ret = torch.addmm(self.bias, x, self.weights) if self.bias is not None else x @ self.weights
        if self.normalizer_fn is not None:
            ret = self.normalizer_fn(ret)
        if self.act_fn is not None:
            ret = self.act_fn(ret)
        return ret


@add_arg_scope
class Upsample(Layer):
    def __init__(self, factor, **kwargs):
        super().__init__(factor=factor, **kwargs)

    def call(self, x):
        return upsample(x, self.factor)


@add_arg_scope
class MaxPool2D(Layer):
    def __init__(self, kernel_size, stride=1, padding="SAME", **kwargs):
        super().__init__(kernel_size=kernel_size, stride=stride, padding=padding, **kwargs)

    def call(self, x):
        x = fix_padding(x, self.kernel_size, padding=self.padding)
        y = F.max_pool2d(x.permute(0, 3, 1, 2), self.kernel_size, self.stride)
        return y.permute(0, 2, 3, 1)
