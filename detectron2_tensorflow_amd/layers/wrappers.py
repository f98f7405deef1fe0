"""Linear / Upsample / MaxPool2D (lib/layers/wrappers.py:13-131)."""
import torch
import torch.nn.functional as F

from ..utils.arg_scope import add_arg_scope
from . import initializers as init
from . import ops
from .activation import get_activation
from .base import Layer
from .convolutional import fix_padding
from .functional import upsample


class _LinearMFMAFn(torch.autograd.Function):
    """x @ w + b as a 1x1 conv over M "pixels" on the split-product MFMA
    kernels: forward d2mi_conv2d_nhwc, dgrad the same kernel with w as the
    transposed conv's packed weights, wgrad + bias gradient one
    d2mi_conv2d_wgrad pass."""

    @staticmethod
    def forward(ctx, x, w, b, packed):
        M, K = x.shape
        N = w.shape[1]
        y = ops.conv2d_nhwc(x.reshape(1, M, 1, K), packed, b, 1, (0, 0))
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return y.reshape(M, N)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        M, K = x.shape
        N = w.shape[1]
        gy4 = gy.contiguous().reshape(1, M, 1, N)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = ops.conv2d_nhwc(gy4, w.detach().reshape(1, 1, K, N).contiguous(), None, 1,
                                 (0, 0)).reshape(M, K)
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            if ctx.has_bias:
                gw, gb = ops.conv2d_wgrad(x.reshape(1, M, 1, K), gy4, 1, with_bias=True)
            else:
                gw = ops.conv2d_wgrad(x.reshape(1, M, 1, K), gy4, 1)
            gw = gw.reshape(K, N)
        return gx, gw, gb, None


class _LinearBiasFn(torch.autograd.Function):
    """torch.addmm(b, x, w) whose backward forms the bias gradient with the
    library's fixed-order column sum (d2mi_column_sum) instead of torch's
    reduction: the weight / input gradients are autograd's own addmm formulas
    (hipBLASLt), but torch's sum over 1,024 rows zeroes its cross-block
    semaphores with a memset, and a memset node inside the graphed step's
    capture is not ordered against the kernels around it while the HIP
    runtime's graph packet capture is on (engine/graphed.py)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return torch.addmm(b, x, w)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = gy.mm(w.t())
        if ctx.needs_input_grad[1]:
            gw = x.t().mm(gy)
        if ctx.needs_input_grad[2]:
            gb = ops.column_sum(gy)
        return gx, gw, gb


@add_arg_scope
class Linear(Layer):
    """x @ weights + bias with weights [in_units, out_units] (TF Dense layout).
    Long-K layers (in_units >= MFMA_MIN_K: the box head's fc1, 12544 -> 1024)
    run on the split-product MFMA conv kernels (fwd / dgrad / wgrad 145 / 134 /
    118 TF/s vs hipBLASLt f32 112 / 90 / 86, tools/exp_linear.py); shorter ones
    (fc2, predictors) on hipBLASLt (torch.addmm), which is faster there."""

    MFMA_MIN_K = 4096

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

    def _packed(self):
        key = (self.weights.data_ptr(), self.weights._version)
        if getattr(self, "_pk_key", None) != key:
            K, N = self.weights.shape
            self._pk = ops.pack_conv_weights(self.weights.detach().reshape(1, 1, K, N))
            self._pk_key = key
        return self._pk

    def call(self, inputs):
        x = inputs.reshape(inputs.shape[0], -1) if inputs.dim() > 2 else inputs
        K, N = self.weights.shape
        if x.is_cuda and K >= self.MFMA_MIN_K and K % 4 == 0 and x.shape[0] > 0:
            ret = _LinearMFMAFn.apply(x.contiguous(), self.weights, self.bias, self._packed())
        elif self.bias is not None and x.is_cuda and torch.is_grad_enabled():
            ret = _LinearBiasFn.apply(x, self.weights, self.bias)
        elif self.bias is not None:
            ret = torch.addmm(self.bias, x, self.weights)
        else:
            ret = x @ self.weights
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
