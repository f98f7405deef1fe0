"""Weight planes (d2mi_conv2d_nhwc_w3 / d2mi_split_bf16x3_many): the split-
product conv kernels reading the step's cached bf16 planes of their weight
operand compute exactly what they compute when they split the f32 weights
themselves -- per kernel configuration (tuning "conv_bp"), per epilogue form,
and through a whole Mask R-CNN training step (the Conv2D forward and the
input-gradient convs of every FoldGroup / PackGroup layer)."""
import os

import pytest
import torch

from test_gpu_train import _cfg

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ops():
    from detectron2_tensorflow_amd.layers import ops as o
    return o


def test_split_bf16x3_many_matches_single(dev):
    g = torch.Generator().manual_seed(3)
    ts = [torch.randn(s, generator=g).to(dev) for s in ((3, 3, 256, 128), (1, 1, 64, 16), (8,))]
    many = ops().split_bf16x3_many(ts)
    for t, m in zip(ts, many):
        assert torch.equal(m, ops().split_bf16x3(t))


@pytest.mark.parametrize("shape", [
    (2, 50, 84, 256, 256, 3),   # warp-specialised 256x128 kernel (cfg 3), split-K
    (2, 30, 40, 256, 256, 1),   # short K: the 3-per-CU 128x128 kernel (cfg 0)
    (2, 30, 40, 256, 64, 1),    # Cout 64: the 128x64 kernel (cfg 1)
    (2, 30, 40, 256, 16, 1),    # Cout 16: the 128x32 kernel (cfg 2)
    (1, 21, 17, 64, 96, 3),     # ragged M / Cout tails
])
def test_conv2d_weight_planes_bit_identical(dev, shape):
    N, H, W, Cin, Cout, k = shape
    pad = (k - 1) // 2
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(N, H, W, Cin, generator=g).to(dev)
    w = (torch.randn(k, k, Cin, Cout, generator=g) / (k * k * Cin) ** 0.5).to(dev)
    b = torch.randn(Cout, generator=g).to(dev)
    res = torch.randn(N, H, W, Cout, generator=g).to(dev)
    gate = torch.randn(N, H, W, Cout, generator=g).to(dev)
    wp = ops().pack_conv_weights(w)
    p3 = ops().split_bf16x3(wp)
    forms = [dict(), dict(relu=True, residual=res, relu_after_add=True),
             dict(residual=res, relu_gate=gate)]
    if k > 1:
        forms.append(dict(flip_taps=True, relu_gate=gate))
    try:
        for bp in (7, 1, 2, 4):
            ops().set_tuning("conv_bp", bp)
            for kw in forms:
                ref = ops().conv2d_nhwc(x, wp, b, 1, (pad, pad), math_mode="split", **kw)
                got = ops().conv2d_nhwc(x, wp, b, 1, (pad, pad), math_mode="split", w_planes=p3,
                                        **kw)
                assert torch.equal(ref, got), (bp, sorted(kw))
    finally:
        ops().set_tuning("conv_bp", 7)


def test_conv2d_planes_only_no_f32_weights(dev):
    """w_packed absent: every configuration reads the planes."""
    from detectron2_tensorflow_amd import _C
    g = torch.Generator().manual_seed(8)
    x = torch.randn(2, 30, 40, 256, generator=g).to(dev)
    w = (torch.randn(1, 1, 256, 256, generator=g) / 16).to(dev)
    wp = ops().pack_conv_weights(w)
    p3 = ops().split_bf16x3(wp)
    ref = ops().conv2d_nhwc(x, wp, None, 1, (0, 0), math_mode="split")
    y = torch.empty_like(ref)
    rc = _C.lib().d2mi_conv2d_nhwc_w3(_C.ptr(x), None, _C.ptr(p3), None, None, None, None,
                                      _C.ptr(y), 2, 30, 40, 256, 256, 1, 1, 1, 0, 0, 4, None, 0,
                                      _C.stream_of(x.device))
    _C.check(rc, "d2mi_conv2d_nhwc_w3")
    assert torch.equal(ref, y)


def test_training_step_with_weight_planes_is_bit_identical(dev, monkeypatch):
    """A Mask R-CNN training step's gradients with the weight planes (every
    trainable FoldGroup / PackGroup conv, forward and input gradient) equal
    those without, bit for bit; the planes engage."""
    from detectron2_tensorflow_amd.layers import convolutional as conv_mod
    from detectron2_tensorflow_amd.modeling import build_model
    from detectron2_tensorflow_amd.utils.synthetic import (calibrate_rcnn_scores,
                                                           synthetic_train_batch)
    cfg = _cfg(True)
    torch.manual_seed(0)
    model = build_model(cfg).to(dev).train()
    batch = synthetic_train_batch(2, 256, 320, 5, dev)
    calibrate_rcnn_scores(model, batch)
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)  # (MIOpen stem)
    used = []
    real = ops().conv2d_nhwc

    def counted(*a, **kw):
        if kw.get("w_planes") is not None:
            used.append(1)
        return real(*a, **kw)

    monkeypatch.setattr(ops(), "conv2d_nhwc", counted)
    grads = {}
    for on in (True, False):
        monkeypatch.setattr(conv_mod.WeightPlanes, "ENABLED", on)
        for m in model.modules():  # drop cached folds / packs / planes
            if isinstance(m, conv_mod.Conv2D):
                m._packed = None
                m.__dict__.pop("_w_planes", None)
        model.zero_grad(set_to_none=True)
        used.clear()
        torch.manual_seed(1)
        losses = model(batch)
        sum(losses.values()).backward()
        assert bool(used) == on
        grads[on] = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    assert grads[True].keys() == grads[False].keys() and grads[True]
    for n in grads[True]:
        assert torch.equal(grads[True][n], grads[False][n]), n
