"""The public op API (lib/layers/__init__.py:1-11) called the way the
reference's own modules call it, through ``detectron2_tensorflow_amd.layers``,
against the CPU oracle:

* ``ROIAlign(output_size, spatial_scale, sampling_ratio, aligned)(x, boxes,
  box_inds)`` (lib/layers/roi_align.py:9-66), sampling_ratio 0 and 2
  (the crop at output x SR + the SR x SR avg pool), aligned and unaligned;
* ``crop_and_resize(image, boxes, box_ind, crop_size, aligned)``
  (lib/layers/functional.py:100-166);
* ``matrix_nms(masks, classes, scores, sum_masks, kernel, sigma)``
  (lib/layers/nms.py:29-83), with and without the caller's sum_masks;
* ``GroupNorm`` with frozen affine parameters still passes the input gradient.
"""
import numpy as np
import pytest
import torch

import oracle
from test_gpu_ops import rand_boxes

pytestmark = pytest.mark.gpu
F32 = np.float32


@pytest.mark.parametrize("sr,aligned", [(0, True), (0, False), (2, True), (2, False)])
def test_roialign_layer_call(dev, sr, aligned):
    from detectron2_tensorflow_amd.layers import ROIAlign
    rng = np.random.default_rng(61)
    x = rng.normal(size=(2, 50, 84, 256)).astype(F32)
    boxes = rand_boxes(rng, 200, 200, 336, 4.0, 300.0)
    inds = rng.integers(0, 2, size=200).astype(np.int32)
    layer = ROIAlign((7, 7), 0.25, sr, aligned)
    got = layer(torch.from_numpy(x).to(dev), torch.from_numpy(boxes).to(dev),
                torch.from_numpy(inds).to(dev)).cpu().numpy()
    want = oracle.roi_align(x, boxes, inds, (7, 7), 0.25, sr, aligned)
    assert got.shape == (200, 7, 7, 256)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-5)


def test_roialign_layer_backward_is_the_adjoint(dev):
    """The layer's input gradient is the adjoint of its forward (through the
    folded SYMMETRIC pad): <ROIAlign(x), g> == <x, dROIAlign^T g> in float64,
    with every row of the forward checked against the oracle first (the
    op-level backward is pinned bit-exact against TF's
    CropAndResizeGradImage in test_gpu_ops.py)."""
    from detectron2_tensorflow_amd.layers import ROIAlign
    rng = np.random.default_rng(62)
    x = rng.normal(size=(1, 40, 60, 64)).astype(F32)
    boxes = rand_boxes(rng, 30, 160, 240, 8.0, 120.0)
    inds = np.zeros(30, np.int32)
    g = rng.normal(size=(30, 7, 7, 64)).astype(F32)
    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    out = ROIAlign((7, 7), 0.25, 0, True)(xt, torch.from_numpy(boxes).to(dev),
                                          torch.from_numpy(inds).to(dev))
    np.testing.assert_allclose(out.detach().cpu().numpy(),
                               oracle.roi_align(x, boxes, inds, (7, 7), 0.25, 0, True), atol=1e-5)
    gt = torch.from_numpy(g).to(dev)
    out.backward(gt)
    lhs = (out.detach().double() * gt.double()).sum().item()
    rhs = (xt.detach().double() * xt.grad.double()).sum().item()
    assert abs(lhs - rhs) <= 1e-5 * max(1.0, abs(lhs))


@pytest.mark.parametrize("aligned", [True, False])
def test_crop_and_resize_functional(dev, aligned):
    from detectron2_tensorflow_amd.layers import crop_and_resize
    rng = np.random.default_rng(63)
    img = rng.normal(size=(3, 64, 96, 32)).astype(F32)
    boxes = rand_boxes(rng, 120, 64, 96, 2.0, 80.0)
    inds = rng.integers(0, 3, size=120).astype(np.int32)
    got = crop_and_resize(torch.from_numpy(img).to(dev), torch.from_numpy(boxes).to(dev),
                          torch.from_numpy(inds).to(dev), (14, 14), aligned).cpu().numpy()
    # crop_and_resize == ROIAlign at spatial_scale 1 with no sampling ratio
    want = oracle.roi_align(img, boxes, inds, (14, 14), 1.0, 0, aligned)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-5)


@pytest.mark.parametrize("kernel", ["gaussian", "linear"])
@pytest.mark.parametrize("given_sums", [False, True])
def test_matrix_nms_layer_api(dev, kernel, given_sums):
    from detectron2_tensorflow_amd.layers import matrix_nms
    rng = np.random.default_rng(64)
    M, H, W = 96, 40, 64
    masks = (rng.uniform(size=(M, H, W)) > 0.6).astype(F32)
    for i in range(0, M - 1, 4):
        masks[i + 1] = np.maximum(masks[i], masks[i + 1] * (rng.uniform() > 0.5))
    classes = rng.integers(0, 5, size=M).astype(np.int32)
    scores = np.sort(rng.uniform(size=M).astype(F32))[::-1].copy()
    sums = masks.reshape(M, -1).sum(1).astype(F32) if given_sums else None
    t = lambda a: torch.from_numpy(a).to(dev)
    got = matrix_nms(t(masks), t(classes), t(scores), t(sums) if given_sums else None,
                     kernel=kernel, sigma=2.0).cpu().numpy()
    want = oracle.matrix_nms(masks, classes, scores, sums, kernel=kernel, sigma=2.0)
    fin = np.isfinite(want)
    np.testing.assert_allclose(got[fin], want[fin], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(got[~fin], want[~fin])
    assert fin.sum() > M // 2


def test_group_norm_frozen_affine_keeps_input_gradient(dev):
    """GroupNorm whose gamma / beta do not train must not take the no-autograd
    HIP path while its input needs a gradient (the upstream convs would lose
    theirs silently)."""
    from detectron2_tensorflow_amd.layers import GroupNorm
    gn = GroupNorm(64, num_groups=16).to(dev)
    gn.gamma.requires_grad_(False)
    gn.beta.requires_grad_(False)
    x = torch.randn(2, 12, 10, 64, device=dev, requires_grad=True)
    assert not gn.fused_ok(x)
    y = gn(x, relu=True)
    g = torch.randn_like(y)
    y.backward(g)
    x2 = x.detach().clone().requires_grad_(True)
    ref = torch.relu(torch.nn.functional.group_norm(x2.permute(0, 3, 1, 2), 16, gn.gamma, gn.beta,
                                                    1e-5).permute(0, 2, 3, 1))
    ref.backward(g)
    assert x.grad is not None
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-6)
    with torch.no_grad():
        assert gn.fused_ok(x)  # inference still takes the HIP kernel
