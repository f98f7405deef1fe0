"""GPU parity tests: every hot-path kernel of libd2mi_hip.so (through the C ABI
via the torch-facing wrappers) against the CPU oracle on the same seeded
inputs and against the committed golden vectors.

Bars (BASELINE.json north_star): kept indices / class ids bit-exact; box
coordinates and features within 1e-4 (absolute, or 2 ulp above 1024 px where
1e-4 is below float32 resolution).
"""
import math
import os

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu
F32 = np.float32
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "nms_golden.npz")


def assert_boxes_close(got, want):
    """|got - want| <= max(1e-4, 2 ulp of the box's largest coordinate): expf is
    not correctly rounded on either side (ocml vs libm / Eigen), and above
    1024 px 1e-4 is below float32 resolution (hard part 3)."""
    got, want = np.asarray(got, F32), np.asarray(want, F32)
    scale = np.abs(want).max(axis=-1, keepdims=True) if want.size else want
    tol = np.maximum(F32(1e-4), 2 * np.spacing(scale.astype(F32)))
    bad = np.abs(got - want) > tol
    assert not bad.any(), f"{bad.sum()} coords off: got {got[bad][:5]} want {want[bad][:5]}"


def ops():
    from detectron2_tensorflow_amd.layers import ops as _ops
    return _ops


def rand_boxes(rng, n, H, W, smin=4.0, smax=None):
    smax = smax or max(H, W) * 0.8
    c = rng.uniform([0, 0], [H, W], size=(n, 2))
    s = np.exp(rng.uniform(np.log(smin), np.log(smax), size=n))
    ar = np.exp(rng.uniform(np.log(0.5), np.log(2.0), size=n))
    h, w = s * np.sqrt(ar), s / np.sqrt(ar)
    return np.stack([c[:, 0] - h / 2, c[:, 1] - w / 2, c[:, 0] + h / 2, c[:, 1] + w / 2], 1).astype(F32)


# ------------------------------------------------------------------ ROIAlign
@pytest.mark.parametrize("C", [64, 6])
def test_roi_align_multilevel_matches_oracle(dev, C):
    rng = np.random.default_rng(1)
    N, IH, IW = 2, 256, 320
    strides = [4, 8, 16, 32]
    feats = [rng.normal(size=(N, IH // s, IW // s, C)).astype(F32) for s in strides]
    boxes = rand_boxes(rng, 300, IH, IW, 2.0, 400.0)
    bimg = rng.integers(0, N, size=300).astype(np.int32)
    scales = [1.0 / s for s in strides]
    for oh in (7, 14):
        want, lv_want = oracle.roi_pooler(feats, boxes, bimg, (oh, oh), scales, 0, True)
        got, lv = ops().roi_align([torch.from_numpy(f).to(dev) for f in feats],
                                  torch.from_numpy(boxes).to(dev), torch.from_numpy(bimg).to(dev),
                                  (oh, oh), scales, 0, True, return_levels=True)
        lv, got = lv.cpu().numpy(), got.cpu().numpy()
        same = lv == lv_want
        np.testing.assert_allclose(got[same], want[same], rtol=0, atol=1e-5)
        # a level differs only for log-boundary boxes (logf rounding on either
        # side), and the GPU's output is the oracle's ROIAlign on its level
        b = boxes.astype(np.float64)
        v = 4 + np.log(np.sqrt((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])) / 224 + 2.0 ** -52) / math.log(2)
        for i in np.nonzero(~same)[0]:
            assert abs(v[i] - round(v[i])) < 1e-5, (i, v[i], lv[i], lv_want[i])
            w1 = oracle.roi_align(feats[lv[i]], boxes[i:i + 1], bimg[i:i + 1], (oh, oh),
                                  scales[lv[i]], 0, True)
            np.testing.assert_allclose(got[i:i + 1], w1, rtol=0, atol=1e-5)


@pytest.mark.parametrize("aligned,sr,pad", [(True, 0, True), (False, 0, True), (True, 2, True),
                                            (False, 2, True), (True, 0, False)])
def test_roi_align_single_level_modes(dev, aligned, sr, pad):
    rng = np.random.default_rng(2)
    img = rng.normal(size=(3, 40, 56, 32)).astype(F32)
    boxes = rand_boxes(rng, 64, 160, 224, 2.0, 300.0)
    boxes[:4] = [[-30, -30, 5, 5], [150, 200, 190, 260], [0, 0, 0, 0], [10, 10, 10.5, 80]]
    bimg = rng.integers(0, 3, size=64).astype(np.int32)
    want = oracle.roi_align(img, boxes, bimg, (7, 7), 0.25, sr, aligned, pad)
    got = ops().roi_align([torch.from_numpy(img).to(dev)], torch.from_numpy(boxes).to(dev),
                          torch.from_numpy(bimg).to(dev), (7, 7), [0.25], sr, aligned, pad)
    np.testing.assert_allclose(got.cpu().numpy(), want, rtol=0, atol=1e-5)


def test_crop_and_resize_raw_mode_matches_tf_semantics(dev):
    rng = np.random.default_rng(3)
    img = rng.normal(size=(2, 17, 23, 8)).astype(F32)
    boxes = rng.uniform(-0.2, 1.2, size=(50, 4)).astype(F32)
    bimg = rng.integers(0, 2, size=50).astype(np.int32)
    for crop in [(5, 9), (1, 1), (28, 28)]:
        want = oracle.crop_and_resize_tf(img, boxes, bimg, crop)
        got = ops().roi_align([torch.from_numpy(img).to(dev)], torch.from_numpy(boxes).to(dev),
                              torch.from_numpy(bimg).to(dev), crop, [1.0], 0, pad_border=False,
                              box_mode=ops().BOX_MODE_RAW)
        np.testing.assert_allclose(got.cpu().numpy(), want, rtol=0, atol=1e-5)


def test_roi_align_backward_raw_matches_tf_grad(dev):
    rng = np.random.default_rng(4)
    img = rng.normal(size=(2, 13, 19, 8)).astype(F32)
    boxes = rng.uniform(-0.1, 1.1, size=(40, 4)).astype(F32)
    bimg = rng.integers(0, 2, size=40).astype(np.int32)
    g = rng.normal(size=(40, 6, 5, 8)).astype(F32)
    want = oracle.crop_and_resize_grad_image(g, boxes, bimg, (2, 13, 19))
    x = torch.from_numpy(img).to(dev).requires_grad_(True)
    out = ops().roi_align([x], torch.from_numpy(boxes).to(dev), torch.from_numpy(bimg).to(dev),
                          (6, 5), [1.0], 0, pad_border=False, box_mode=ops().BOX_MODE_RAW)
    out.backward(torch.from_numpy(g).to(dev))
    # the tiled gather sums each pixel in the TF kernel's (box, y, x, corner) order
    np.testing.assert_array_equal(x.grad.cpu().numpy(), want)


def test_roi_align_backward_unaligned_grad_maps(dev):
    """d2mi_roi_align_bwd on caller-owned gradient maps that start 4 B past a
    16-B boundary (a sliced tensor): the clear kernel's unaligned head and
    tail paths.  Untouched pixels come back zero, touched ones equal the TF
    CropAndResizeGradImage restatement, and the guard words around the maps
    are not written."""
    from detectron2_tensorflow_amd import _C
    rng = np.random.default_rng(44)
    N, H, W, C, R, oh, ow = 2, 13, 19, 8, 40, 6, 5
    boxes = rng.uniform(-0.1, 0.9, size=(R, 4)).astype(F32)
    bimg = rng.integers(0, N, size=R).astype(np.int32)
    g = rng.normal(size=(R, oh, ow, C)).astype(F32)
    want = oracle.crop_and_resize_grad_image(g, boxes, bimg, (N, H, W))
    n = N * H * W * C
    buf = torch.full((n + 2,), 7.0, dtype=torch.float32, device=dev)  # guard word each side
    grad = buf[1:n + 1]
    assert grad.data_ptr() % 16 == 4
    bt, it, gt = (torch.from_numpy(boxes).to(dev), torch.from_numpy(bimg).to(dev),
                  torch.from_numpy(g).to(dev))
    gp = _C.host_array(_C.c_void_p, [grad.data_ptr()])
    dims = _C.host_array(_C.ctypes.c_int32, [N, H, W])
    sc = _C.host_array(_C.c_float, [1.0])
    wsb = _C.lib().d2mi_roi_align_bwd_workspace_size(dims, 1, C, R, oh, ow, 0)
    ws = _C.workspace(wsb, dev)
    rc = _C.lib().d2mi_roi_align_bwd(gp, dims, sc, 1, C, _C.ptr(bt), _C.ptr(it), R, oh, ow, 0,
                                     ops().BOX_MODE_RAW, 0, 0, 0, 0, 224, 4, _C.ptr(gt),
                                     _C.ptr(ws), wsb, _C.stream_of(dev))
    _C.check(rc, "d2mi_roi_align_bwd")
    got = buf.cpu().numpy()
    assert got[0] == 7.0 and got[-1] == 7.0
    np.testing.assert_array_equal(got[1:n + 1].reshape(N, H, W, C), want)
    assert (want == 0).any()  # some pixels untouched: the clear path is exercised


@pytest.mark.parametrize("C,crop,sr", [(300, (14, 14), 0), (64, (7, 7), 2), (3, (28, 20), 0)])
def test_roi_align_backward_raw_large_crops_and_ragged_channels(dev, C, crop, sr):
    """More samples than one 64-lane block, channel counts off the 64-chunk grid,
    boxes spanning many 8x8 tiles (and flipped ones)."""
    rng = np.random.default_rng(C)
    img = rng.normal(size=(3, 40, 52, C)).astype(F32)
    boxes = rng.uniform(-0.2, 1.2, size=(25, 4)).astype(F32)
    bimg = rng.integers(0, 3, size=25).astype(np.int32)
    x = torch.from_numpy(img).to(dev).requires_grad_(True)
    out = ops().roi_align([x], torch.from_numpy(boxes).to(dev), torch.from_numpy(bimg).to(dev),
                          crop, [1.0], sr, pad_border=False, box_mode=ops().BOX_MODE_RAW)
    g = rng.normal(size=tuple(out.shape)).astype(F32)
    out.backward(torch.from_numpy(g).to(dev))
    if sr == 0:
        # pixels with > 64 contributions are summed as 64-long partials: not bit-exact
        want = oracle.crop_and_resize_grad_image(g, boxes, bimg, (3, 40, 52))
        np.testing.assert_allclose(x.grad.cpu().numpy(), want, rtol=1e-5, atol=1e-5)
    else:
        lhs = (out.double() * torch.from_numpy(g).to(dev).double()).sum().item()
        rhs = (x.double() * x.grad.double()).sum().item()
        assert abs(lhs - rhs) <= 1e-4 * max(1.0, abs(lhs))


@pytest.mark.parametrize("heavy", [16, 1, 0])
@pytest.mark.parametrize("C,sr", [(256, 2), (256, 3), (256, 1), (64, 2)])
def test_roi_align_backward_sampled_bins_bit_exact(dev, C, sr, heavy):
    """Sampling ratio > 0 (the poolers' mode): TF's backward is AvgPoolGrad
    (each bin's gradient / sr^2 to its sr x sr samples) then
    CropAndResizeGradImage over the sr-times-finer crop -- bit-exact, also
    where sr^2 is a power of two and the kernels multiply by its reciprocal
    instead of dividing (C = 256: the four-pixels-per-wave pass)."""
    from detectron2_tensorflow_amd.layers import ops as lops
    old_heavy = lops.get_tuning("roi_heavy")  # touched-list order: heavy pixels first (> heavy)
    lops.set_tuning("roi_heavy", heavy)
    try:
        _sampled_bins_case(dev, C, sr)
    finally:
        lops.set_tuning("roi_heavy", old_heavy)


def _sampled_bins_case(dev, C, sr):
    rng = np.random.default_rng(100 + sr)
    img = rng.normal(size=(2, 23, 29, C)).astype(F32)
    lo = rng.uniform(0.0, 0.3, size=(12, 2))
    boxes = np.concatenate([lo, lo + rng.uniform(0.5, 0.7, size=(12, 2))], 1)[:, [0, 1, 2, 3]]
    boxes = boxes.astype(F32)
    bimg = rng.integers(0, 2, size=12).astype(np.int32)
    x = torch.from_numpy(img).to(dev).requires_grad_(True)
    out = ops().roi_align([x], torch.from_numpy(boxes).to(dev), torch.from_numpy(bimg).to(dev),
                          (7, 7), [1.0], sr, pad_border=False, box_mode=ops().BOX_MODE_RAW)
    g = rng.normal(size=tuple(out.shape)).astype(F32)
    out.backward(torch.from_numpy(g).to(dev))
    gs = (g / F32(sr * sr)).astype(F32)
    up = np.repeat(np.repeat(gs, sr, axis=1), sr, axis=2)
    want = oracle.crop_and_resize_grad_image(up, boxes, bimg, (2, 23, 29))
    np.testing.assert_array_equal(x.grad.cpu().numpy(), want)


def test_roi_align_backward_hot_pixels(dev):
    """Hundreds of ROIs collapsed onto the same pixels (degenerate proposals at
    the border): the split-segment path, against the TF scatter."""
    rng = np.random.default_rng(9)
    img = rng.normal(size=(2, 24, 30, 64)).astype(F32)
    boxes = np.concatenate([np.tile([[0.5, 0.5, 0.5, 0.5]], (300, 1)),
                            rng.uniform(0, 1, size=(50, 4))]).astype(F32)
    bimg = np.concatenate([np.zeros(300), rng.integers(0, 2, 50)]).astype(np.int32)
    x = torch.from_numpy(img).to(dev).requires_grad_(True)
    out = ops().roi_align([x], torch.from_numpy(boxes).to(dev), torch.from_numpy(bimg).to(dev),
                          (7, 7), [1.0], 0, pad_border=False, box_mode=ops().BOX_MODE_RAW)
    g = rng.normal(size=tuple(out.shape)).astype(F32)
    out.backward(torch.from_numpy(g).to(dev))
    want = oracle.crop_and_resize_grad_image(g, boxes, bimg, (2, 24, 30))
    got = x.grad.cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-3)
    x.grad = None
    out = ops().roi_align([x], torch.from_numpy(boxes).to(dev), torch.from_numpy(bimg).to(dev),
                          (7, 7), [1.0], 0, pad_border=False, box_mode=ops().BOX_MODE_RAW)
    out.backward(torch.from_numpy(g).to(dev))
    assert np.array_equal(x.grad.cpu().numpy(), got)


def test_roi_align_backward_is_deterministic(dev):
    rng = np.random.default_rng(11)
    strides = [4, 8, 16, 32]
    feats = [torch.from_numpy(rng.normal(size=(2, 256 // s, 320 // s, 256)).astype(F32)).to(dev)
             .requires_grad_(True) for s in strides]
    boxes = torch.from_numpy(rand_boxes(rng, 512, 256, 320, 2, 300)).to(dev)
    bimg = torch.from_numpy(rng.integers(0, 2, size=512).astype(np.int32)).to(dev)
    g = torch.randn(512, 7, 7, 256, device=dev)
    runs = []
    for _ in range(2):
        for f in feats:
            f.grad = None
        out = ops().roi_align(feats, boxes, bimg, (7, 7), [1.0 / s for s in strides], 0, True)
        out.backward(g)
        runs.append([f.grad.clone() for f in feats])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def test_roi_align_backward_is_adjoint_multilevel(dev):
    """<roi_align(x), g> == <x, roi_align^T(g)> for the padded, aligned, SR=2 pooler."""
    rng = np.random.default_rng(5)
    strides = [4, 8, 16, 32]
    feats = [torch.from_numpy(rng.normal(size=(2, 128 // s, 160 // s, 16)).astype(F32)).to(dev)
             .requires_grad_(True) for s in strides]
    boxes = torch.from_numpy(rand_boxes(rng, 100, 128, 160, 2, 200)).to(dev)
    bimg = torch.from_numpy(rng.integers(0, 2, size=100).astype(np.int32)).to(dev)
    out = ops().roi_align(feats, boxes, bimg, (7, 7), [1.0 / s for s in strides], 2, True)
    g = torch.randn_like(out)
    (out * g).sum().backward()
    lhs = (out.double() * g.double()).sum().item()
    rhs = sum((f.double() * f.grad.double()).sum().item() for f in feats)
    assert abs(lhs - rhs) <= 1e-4 * max(1.0, abs(lhs))


def test_roi_align_bad_box_index_sets_error_word(dev):
    from detectron2_tensorflow_amd import _C
    _C.clear_errors()
    img = torch.zeros(1, 8, 8, 4, device=dev)
    out = ops().roi_align([img], torch.tensor([[0, 0, 4, 4.0]], device=dev),
                          torch.tensor([3], dtype=torch.int32, device=dev), (2, 2), [1.0])
    assert torch.all(out == 0)
    with pytest.raises(_C.D2MIError, match="box index"):
        _C.raise_on_errors()


# ----------------------------------------------------------------------- NMS
def test_nms_golden_reference_vectors(dev):
    """d2mi_nms reproduces the reference numpy NMS goldens, all cases batched
    into one segmented launch per (threshold, max_out) group."""
    d = np.load(GOLDEN)
    for i in range(int(d["num_cases"])):
        thr, max_out = d[f"c{i}_params"]
        b, s = d[f"c{i}_boxes"], d[f"c{i}_scores"]
        keep = ops().non_max_suppression(torch.from_numpy(b).to(dev), torch.from_numpy(s).to(dev),
                                         int(max_out), float(thr))
        np.testing.assert_array_equal(keep.cpu().numpy(), d[f"c{i}_keep"], err_msg=f"case {i}")


@pytest.fixture(params=[1, 0], ids=["scan_fixed_point", "scan_serial"])
def nms_scan(request):
    """Both NMS scans (tuning "nms_scan": 1 the r5 fixed-point tile resolve,
    0 the serial one), restored after the test."""
    from detectron2_tensorflow_amd.layers import ops as lops
    old = lops.get_tuning("nms_scan")
    lops.set_tuning("nms_scan", request.param)
    yield request.param
    lops.set_tuning("nms_scan", old)


@pytest.mark.parametrize("thr", [0.0, 0.3, 0.5, 0.7, 1.0])
def test_nms_segmented_vs_oracle_with_ties(dev, thr, nms_scan):
    rng = np.random.default_rng(int(thr * 10) + 7)
    lens = [0, 1, 5, 64, 65, 200, 1000, 2000, 777]
    boxes, scores, off = [], [], [0]
    for n in lens:
        b = rand_boxes(rng, n, 300, 300, 4, 120)
        if n > 10:
            b[: n // 10] = b[n // 10: 2 * (n // 10)]           # exact duplicates
            b[-3:] = b[-3:, [2, 3, 0, 1]]                      # flipped corners
        s = np.round(rng.uniform(0, 1, size=n), 2).astype(F32)  # many ties
        if n > 3:
            s[0] = np.nan
            s[1] = -np.inf
        boxes.append(b)
        scores.append(s)
        off.append(off[-1] + n)
    boxes, scores, off = np.concatenate(boxes), np.concatenate(scores), np.array(off, np.int32)
    for max_out in (1, 100, 1000):
        want_k, want_n = oracle.nms_batched(boxes, scores, off, max_out, thr)
        k, n = ops().nms_segments(torch.from_numpy(boxes).to(dev), torch.from_numpy(scores).to(dev),
                                  torch.from_numpy(off).to(dev), max_out, thr,
                                  seg_capacity=max(lens))
        np.testing.assert_array_equal(n.cpu().numpy(), want_n)
        np.testing.assert_array_equal(k.cpu().numpy(), want_k)


@pytest.mark.parametrize("thr", [0.5, 0.7, 0.3])
def test_nms_iou_at_the_threshold_is_exact(dev, thr, nms_scan):
    """Box pairs whose IoU is the threshold to within a few ulps -- exactly
    equal (not suppressed: TF's test is IoU > thr), a few ulps either side,
    and random shapes at the threshold up to their coordinates' rounding: the
    float32 quotient's rounding decides every pair, and the kept sets equal
    the oracle's.  (r6 measured a division-free form of this test -- a
    reciprocal estimate outside a 2^-18 margin, exact by construction and
    green here -- at no gain in the RetinaNet or training step,
    profiles/r6ay_iou_fast_ab.txt, and did not keep it.)"""
    rng = np.random.default_rng(int(thr * 100))
    pairs = []
    # IoU of [y, x, y + h, x + w] and [y, x + dx, y + h, x + w + dx] is
    # (w - dx) / (w + dx): integer w = a m, dx = b m with (a - b) / (a + b) =
    # thr hit the threshold's float exactly; the second box's x corners then
    # move 0 .. 3 ulps either way (IoU a few ulps off the threshold)
    a, b = {0.5: (3, 1), 0.7: (17, 3), 0.3: (13, 7)}[thr]
    for _ in range(2000):
        m = int(rng.integers(1, 12))
        h, w, dx = F32(rng.integers(1, 200)), F32(a * m), F32(b * m)
        y0, x0 = F32(rng.integers(0, 4000)), F32(rng.integers(0, 4000))
        x1, x2 = F32(x0 + dx), F32(x0 + w + dx)
        for _k in range(int(rng.integers(0, 4))):
            step = np.inf if rng.integers(0, 2) else -np.inf
            x1, x2 = np.nextafter(x1, F32(step)), np.nextafter(x2, F32(-step))
        pairs.append([[y0, x0, y0 + h, x0 + w], [y0, x1, y0 + h, x2]])
    # and random shapes at the threshold up to the coordinates' rounding
    for _ in range(1000):
        h, w = F32(rng.uniform(1, 200)), F32(rng.uniform(1, 200))
        dx = F32(w * (1 - thr) / (1 + thr))
        y0, x0 = F32(rng.uniform(0, 5000)), F32(rng.uniform(0, 5000))
        pairs.append([[y0, x0, y0 + h, x0 + w], [y0, x0 + dx, y0 + h, x0 + w + dx]])
    boxes = np.asarray(pairs, F32).reshape(-1, 4)
    n = boxes.shape[0]
    scores = np.linspace(1.0, 0.0, n, dtype=F32)
    lens = [64, 1000, 2000, n - 3064]  # several segments, the same pairs order
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    want_k, want_n = oracle.nms_batched(boxes, scores, off, 2000, thr)
    k, m = ops().nms_segments(torch.from_numpy(boxes).to(dev), torch.from_numpy(scores).to(dev),
                              torch.from_numpy(off).to(dev), 2000, thr, seg_capacity=max(lens))
    np.testing.assert_array_equal(m.cpu().numpy(), want_n)
    np.testing.assert_array_equal(k.cpu().numpy(), want_k)
    # the pairs do straddle the threshold: some second boxes kept, some not
    kept = int(want_n.sum())
    assert n // 2 < kept < n, kept


@pytest.mark.parametrize("cap", [2000, 4096, 4160])
def test_nms_suppression_chains_and_truncation(dev, cap, nms_scan):
    """Chains of boxes each overlapping the next above the threshold (the
    greedy keeps every other one: the fixed-point resolve's worst case, one
    round per row of a tile) next to clusters and random boxes; max_out cuts
    inside a tile; capacity 4,096 is the fixed-point scan's largest (64 tiles),
    4,160 falls back to the serial scan."""
    rng = np.random.default_rng(cap)
    segs = []
    chain = np.array([[0, 10 * i, 100, 10 * i + 100] for i in range(cap // 2)], F32)
    segs.append((chain, np.linspace(1, 0.1, len(chain)).astype(F32)))
    n = cap
    b = rand_boxes(rng, n, 600, 600, 4, 200)
    b[: n // 4] = np.array([[5, 5, 105, 105]], F32) + rng.uniform(0, 8, size=(n // 4, 1)).astype(F32)
    segs.append((b, rng.uniform(size=n).astype(F32)))
    segs.append((rand_boxes(rng, 777, 300, 300, 4, 120), rng.uniform(size=777).astype(F32)))
    boxes = np.concatenate([x for x, _ in segs])
    scores = np.concatenate([y for _, y in segs])
    off = np.cumsum([0] + [len(y) for _, y in segs]).astype(np.int32)
    for thr, max_out in ((0.5, 1000), (0.5, 37), (0.7, 5000), (0.05, 99)):
        want_k, want_n = oracle.nms_batched(boxes, scores, off, max_out, thr)
        k, nk = ops().nms_segments(torch.from_numpy(boxes).to(dev),
                                   torch.from_numpy(scores).to(dev), torch.from_numpy(off).to(dev),
                                   max_out, thr, seg_capacity=cap)
        np.testing.assert_array_equal(nk.cpu().numpy(), want_n)
        np.testing.assert_array_equal(k.cpu().numpy(), want_k)


@pytest.mark.parametrize("n,tied", [(12000, False), (40000, True), (70001, False)])
def test_nms_large_segment_uses_radix_sort_path(dev, n, tied):
    """Segments over 8,192 candidates: the hand-written tile rank sort + merge
    passes (csrc/sort.hip; r1-r3 ran rocPRIM's radix sort here) -- 2, 5 and 9
    tiles (an odd run count, up to 4 merge passes), heavy score ties (order
    by index) and NaN / -inf scores (never selected)."""
    rng = np.random.default_rng(11 + n)
    b = rand_boxes(rng, n, 1000, 1300, 8, 300)
    s = rng.uniform(size=n).astype(F32)
    if tied:
        s = np.round(s * 50) / 50
        s[::97] = np.nan
        s[5::89] = -np.inf
    want = oracle.nms(b, s, 300, 0.5)
    got = ops().non_max_suppression(torch.from_numpy(b).to(dev), torch.from_numpy(s).to(dev), 300, 0.5)
    np.testing.assert_array_equal(got.cpu().numpy(), want)


# --------------------------------------------------------------------- top-k
def test_topk_segments_vs_oracle(dev):
    rng = np.random.default_rng(12)
    lens = [1, 10, 999, 5000, 9000, 201600, 300000, 300001, 1 << 20, 3001]
    vals = [rng.normal(size=n).astype(F32) for n in lens]
    # signed zeros: -0.0 ties +0.0 (the index decides) and comes back as -0.0
    vals[9] = np.round(vals[9] * 0.6).astype(F32)
    vals[9][(vals[9] == 0) & (rng.uniform(size=lens[9]) < 0.5)] = -0.0
    vals[3] = np.round(vals[3], 1)           # heavy ties
    vals[4][:] = 0.5                          # all tied: ordered-ties path
    vals[6] = np.round(vals[6] * 4) / 4       # ties straddling the threshold bin
    # saturated logits: every sigmoid is exactly 1.0 (both sides), so key_mode 1
    # takes the ordered path over the sigmoid tie group (lowest indices first)
    # while the raw values are all distinct; odd length + odd start (unaligned)
    vals[7] = np.maximum(rng.normal(40, 5, size=lens[7]), 25).astype(F32)
    vals[8] = (rng.normal(-3, 1, size=lens[8])).astype(F32)  # RetinaNet-like, big-chunk path
    flat = np.concatenate(vals)
    start = np.cumsum([0] + lens[:-1]).astype(np.int64)
    for k in (1, 1000, 2000):
        for sig in (False, True):
            v, i, c = ops().topk_segments(torch.from_numpy(flat).to(dev),
                                          torch.from_numpy(start).to(dev),
                                          torch.tensor(lens, dtype=torch.int32, device=dev), k,
                                          max(lens), sigmoid=sig)
            v, i, c = v.cpu().numpy(), i.cpu().numpy(), c.cpu().numpy()
            for s, x in enumerate(vals):
                key = oracle.sigmoid(x) if sig else x
                wv, wi = oracle.top_k(key, k)
                assert c[s] == len(wi)
                if sig:
                    # GPU expf vs CPU expf may differ by 1 ulp: compare values,
                    # and indices on the saturated segment (exact ties at 1.0)
                    np.testing.assert_allclose(v[s, : c[s]], wv, rtol=1e-6, atol=0)
                    if s == 7:
                        assert (wv == 1.0).all()
                        np.testing.assert_array_equal(i[s, : c[s]], wi)
                else:
                    np.testing.assert_array_equal(i[s, : c[s]], wi)
                    np.testing.assert_array_equal(v[s, : c[s]].view(np.int32),
                                                  np.asarray(wv, F32).view(np.int32))


# ------------------------------------------------------------ anchors/deltas
def test_grid_anchors_and_apply_deltas_vs_oracle(dev):
    cell = oracle.generate_cell_anchors([32 * 2 ** (1 / 3)], [0.5, 1.0, 2.0])
    got = ops().grid_anchors(13, 21, 8, torch.from_numpy(cell), dev).cpu().numpy()
    np.testing.assert_array_equal(got, oracle.grid_anchors(13, 21, 8, cell))
    rng = np.random.default_rng(13)
    boxes = rand_boxes(rng, 500, 800, 1333)
    d = rng.normal(0, 1.5, size=(500, 80 * 4)).astype(F32)
    d[0, 2] = 50.0  # clamp path
    for w in [(10, 10, 5, 5), (1, 1, 1, 1)]:
        want = oracle.apply_deltas(d, boxes, w)
        got = ops().apply_deltas(torch.from_numpy(d).to(dev), torch.from_numpy(boxes).to(dev), w)
        assert_boxes_close(got.cpu().numpy().reshape(-1, 4), want.reshape(-1, 4))


# ------------------------------------------------------------ RPN proposals
def _rpn_case(seed, N=2, IH=256, IW=320, A=3):
    rng = np.random.default_rng(seed)
    strides = [4, 8, 16, 32, 64]
    hw = [(int(math.ceil(IH / s)), int(math.ceil(IW / s))) for s in strides]
    cells = [oracle.generate_cell_anchors([sz], [0.5, 1.0, 2.0]) for sz in [32, 64, 128, 256, 512]]
    logits = [rng.normal(size=(N, h, w, A)).astype(F32) for h, w in hw]
    deltas = [rng.normal(0, 0.3, size=(N, h, w, A * 4)).astype(F32) for h, w in hw]
    image_hw = np.array([[IH - 17, IW], [IH, IW - 40]], np.int32)[:N]
    return strides, hw, cells, logits, deltas, image_hw


@pytest.mark.parametrize("merge,compact", [(1, 1), (0, 1), (1, 0)])
@pytest.mark.parametrize("tied", [False, True])
@pytest.mark.parametrize("pre,post,min_size", [(1000, 1000, 0.0), (300, 200, 0.0), (1000, 500, 8.0)])
def test_rpn_proposals_vs_oracle(dev, pre, post, min_size, tied, merge, compact):
    """merge: the per-image concat + top-k as a merge rank over the per-level
    survivor lists (tuning "rpn_merge" 1, r5) or one workgroup's bitonic sort
    (0).  compact: decode + a stable compaction of the valid top-k entries as
    the NMS input (tuning "rpn_compact" 1, r5) or decode -> keys -> the NMS's
    own sort (0).  tied: logits quantized to halves with signed zeros, so
    equal scores across levels exercise the level-then-position tie rule (-0
    tied with +0: the index decides)."""
    from detectron2_tensorflow_amd.layers import ops as lops
    strides, hw, cells, logits, deltas, image_hw = _rpn_case(21)
    if tied:
        logits = [np.round(l * 2) / 2 for l in logits]
        for l in logits:
            l[..., 0][np.abs(l[..., 0]) < 0.25] = -0.0
        logits = [l.astype(F32) for l in logits]
    old = lops.get_tuning("rpn_merge"), lops.get_tuning("rpn_compact")
    lops.set_tuning("rpn_merge", merge)
    lops.set_tuning("rpn_compact", compact)
    try:
        _rpn_proposals_vs_oracle(dev, pre, post, min_size, strides, hw, cells, logits, deltas,
                                 image_hw)
    finally:
        lops.set_tuning("rpn_merge", old[0])
        lops.set_tuning("rpn_compact", old[1])


def _rpn_proposals_vs_oracle(dev, pre, post, min_size, strides, hw, cells, logits, deltas,
                             image_hw):
    N = logits[0].shape[0]
    props = []
    for (h, w), s, c, d in zip(hw, strides, cells, deltas):
        anc = oracle.grid_anchors(h, w, s, c)
        props.append(oracle.apply_deltas(d.reshape(-1, 4), np.tile(anc, (N, 1)), (1, 1, 1, 1))
                     .reshape(N, -1, 4))
    wb, ws, wv = oracle.find_top_rpn_proposals(props, [l.reshape(N, -1) for l in logits],
                                               image_hw, 0.7, pre, post, min_size)
    gb, gs, gv = ops().rpn_proposals([torch.from_numpy(l).to(dev) for l in logits],
                                     [torch.from_numpy(d).to(dev) for d in deltas], strides,
                                     [torch.from_numpy(c) for c in cells],
                                     torch.from_numpy(image_hw).to(dev), pre, post, 0.7, min_size)
    np.testing.assert_array_equal(gv.cpu().numpy(), wv)
    np.testing.assert_array_equal(gs.cpu().numpy(), ws)
    # bit for bit: a -0.0 logit stays a -0.0 score (TF's top_k returns the
    # input value; assert_array_equal alone treats the two zeros as equal)
    np.testing.assert_array_equal(gs.cpu().numpy().view(np.int32), ws.astype(F32).view(np.int32))
    assert_boxes_close(gb.cpu().numpy(), wb)


# ------------------------------------------------------------- Fast R-CNN
def test_fast_rcnn_inference_vs_oracle(dev):
    rng = np.random.default_rng(31)
    N, P, K = 2, 300, 80
    image_hw = np.array([[800, 1333], [640, 1000]], np.int32)
    counts = [300, 217]
    roi_img = np.concatenate([np.full(c, n) for n, c in enumerate(counts)]).astype(np.int32)
    roi_slot = np.concatenate([np.arange(c) for c in counts]).astype(np.int32)
    R = len(roi_img)
    props = np.concatenate([rand_boxes(rng, c, *image_hw[n]) for n, c in enumerate(counts)])
    logits = rng.normal(0, 3, size=(R, K + 1)).astype(F32)
    deltas = rng.normal(0, 0.5, size=(R, K * 4)).astype(F32)
    w = (10.0, 10.0, 5.0, 5.0)
    probs = oracle.softmax(logits)
    boxes = oracle.apply_deltas(deltas, props, w)
    want = oracle.fast_rcnn_inference(boxes, probs, roi_img, roi_slot, P, image_hw, 0.05, 0.5, 100)
    gb, gs, gc, gv, groi = ops().fast_rcnn_inference(
        torch.from_numpy(logits).to(dev), torch.from_numpy(deltas).to(dev),
        torch.from_numpy(props).to(dev), torch.from_numpy(roi_img).to(dev),
        torch.from_numpy(roi_slot).to(dev), N, P, torch.from_numpy(image_hw).to(dev), w, 0.05,
        0.5, 100)
    for n in range(N):
        wb, wsc, wc, wv, wroi = want[n]
        np.testing.assert_array_equal(gv[n].cpu().numpy(), wv)
        np.testing.assert_array_equal(gc[n].cpu().numpy(), wc)
        np.testing.assert_array_equal(groi[n].cpu().numpy(), wroi)
        np.testing.assert_allclose(gs[n].cpu().numpy(), wsc, rtol=2e-6, atol=1e-7)
        assert_boxes_close(gb[n].cpu().numpy(), wb)


def test_fast_rcnn_inference_dense_layout_ignores_negative_slots(dev):
    """The model's dense [N, P] layout: padded rows carry roi_slot = -1 and are
    skipped without raising the error word."""
    from detectron2_tensorflow_amd import _C
    rng = np.random.default_rng(32)
    N, P, K = 2, 200, 80
    image_hw = np.array([[800, 1333], [640, 1000]], np.int32)
    valid = np.ones((N, P), bool)
    valid[1, 150:] = False
    roi_img = np.repeat(np.arange(N), P).astype(np.int32)
    roi_slot = np.where(valid.reshape(-1), np.tile(np.arange(P), N), -1).astype(np.int32)
    props = np.concatenate([rand_boxes(rng, P, *image_hw[n]) for n in range(N)])
    logits = rng.normal(0, 3, size=(N * P, K + 1)).astype(F32)
    deltas = rng.normal(0, 0.5, size=(N * P, K * 4)).astype(F32)
    w = (10.0, 10.0, 5.0, 5.0)
    keep = valid.reshape(-1)
    want = oracle.fast_rcnn_inference(oracle.apply_deltas(deltas[keep], props[keep], w),
                                      oracle.softmax(logits[keep]), roi_img[keep], roi_slot[keep],
                                      P, image_hw, 0.05, 0.5, 100)
    _C.clear_errors()
    t = lambda a: torch.from_numpy(a).to(dev)
    gb, gs, gc, gv, groi = ops().fast_rcnn_inference(t(logits), t(deltas), t(props), t(roi_img),
                                                      t(roi_slot), N, P, t(image_hw), w, 0.05,
                                                      0.5, 100)
    _C.raise_on_errors(dev)
    for n in range(N):
        wb, wsc, wc, wv, wroi = want[n]
        np.testing.assert_array_equal(gv[n].cpu().numpy(), wv)
        np.testing.assert_array_equal(gc[n].cpu().numpy(), wc)
        np.testing.assert_allclose(gs[n].cpu().numpy(), wsc, rtol=2e-6, atol=1e-7)
        assert_boxes_close(gb[n].cpu().numpy(), wb)


# -------------------------------------------------------------- RetinaNet
def assert_sigmoid_scores_close(got, want):
    """Sigmoid scores 1 / (1 + expf(-x)): ocml's expf and libm's differ by up to
    1 ulp, which the add and the divide carry to at most 2 ulp of the score."""
    got, want = np.asarray(got, F32), np.asarray(want, F32)
    assert got.shape == want.shape
    bad = np.abs(got.astype(np.float64) - want) > 2 * np.spacing(np.abs(want)).astype(np.float64)
    assert not bad.any(), (got[bad][:5], want[bad][:5])


def _retina_logits(rng, shape, dist):
    x = rng.normal(-3, 1, size=shape)
    if dist == "quantized":  # big tie groups at every value, some on the sampled floor
        x = np.round(x * 4) / 4
    elif dist == "saturated":  # >8192 keys with sigmoid == 1.0: floor overflows -> radix passes
        x = np.where(rng.uniform(size=shape) < 0.2, rng.uniform(20, 40, size=shape), x)
    elif dist == "sparse":  # few scores above 0.05: top-k mostly filtered
        x = x - 3
    return x.astype(F32)


@pytest.mark.parametrize("path", ["fused", "fused_exact_select", "fused_rank_inline", "fused_r5",
                                  "fused_rank_windowed", "unfused"])
@pytest.mark.parametrize("dist", ["normal", "quantized", "saturated", "sparse"])
def test_retinanet_inference_vs_oracle(dev, dist, path):
    """Dense top-k + decode + NMS vs the oracle.  The distributions drive the
    top-k down both of its paths: the sampled floor (normal, quantized, sparse)
    and the exact select it falls back to (saturated: the tie group of
    sigmoid == 1 overflows the candidate buffer).  ``path``: the four-launch
    pipeline (csrc/retina_post.hip, tuning "retina_fused" = 1), the same with
    its in-workgroup exact select forced on every level (2), the same with the
    merge rank inside the NMS workgroup (tuning "retina_rank" = 1; default: its
    own launch), the r5 form (tuning "retina_var" = 0; the default 12018
    compacts the wave slots with many workgroups before the finish, stops the
    finish's select at the first bound leaving <= 1,024 keys, runs its bitonic
    exchanges, reductions and scans in DPP / permlane lane permutations,
    computes the NMS IoU only where the boxes intersect, resolves each NMS
    tile as a ballot fixed point, selects the floor by a workgroup radix
    select spreading a small level's samples over the level, and loops the
    rank launch's rounds), the same with the merge rank
    windowed inside the NMS (16080), and the unfused top-k / sort / mask NMS
    pipeline (0)."""
    from detectron2_tensorflow_amd.layers import ops as lops
    old = lops.get_tuning("retina_fused")
    old_rank = lops.get_tuning("retina_rank")
    old_var = lops.get_tuning("retina_var")
    lops.set_tuning("retina_fused", {"fused": 1, "fused_exact_select": 2, "fused_rank_inline": 1,
                                     "fused_r5": 1, "fused_rank_windowed": 1, "unfused": 0}[path])
    lops.set_tuning("retina_rank", 1 if path == "fused_rank_inline" else 0)
    lops.set_tuning("retina_var", {"fused_r5": 0, "fused_rank_windowed": 16080}.get(path, old_var))
    try:
        _retinanet_inference_vs_oracle(dev, dist)
    finally:
        lops.set_tuning("retina_fused", old)
        lops.set_tuning("retina_rank", old_rank)
        lops.set_tuning("retina_var", old_var)


def _retinanet_inference_vs_oracle(dev, dist):
    rng = np.random.default_rng(41)
    N, IH, IW, A, K = 2, 320, 320, 9, 80
    strides = [8, 16, 32, 64, 128]
    hw = [(int(math.ceil(IH / s)), int(math.ceil(IW / s))) for s in strides]
    cells = [oracle.generate_cell_anchors([x, x * 2 ** (1 / 3), x * 2 ** (2 / 3)], [0.5, 1.0, 2.0])
             for x in [32, 64, 128, 256, 512]]
    cls = [_retina_logits(rng, (N, h, w, A * K), dist) for h, w in hw]
    box = [rng.normal(0, 0.3, size=(N, h, w, A * 4)).astype(F32) for h, w in hw]
    anchors = [oracle.grid_anchors(h, w, s, c) for (h, w), s, c in zip(hw, strides, cells)]
    want = oracle.retinanet_inference([c.reshape(N, -1, K) for c in cls],
                                      [b.reshape(N, -1, 4) for b in box], anchors, K, 1000, 0.05,
                                      0.5, 100, (1, 1, 1, 1))
    gb, gs, gc, gv = ops().retinanet_inference([torch.from_numpy(c).to(dev) for c in cls],
                                               [torch.from_numpy(b).to(dev) for b in box], strides,
                                               [torch.from_numpy(c) for c in cells], K, 1000, 0.05,
                                               0.5, 100)
    for n in range(N):
        wb, wsc, wc, wv = want[n]
        np.testing.assert_array_equal(gv[n].cpu().numpy(), wv)
        np.testing.assert_array_equal(gc[n].cpu().numpy(), wc)
        assert_sigmoid_scores_close(gs[n].cpu().numpy(), wsc)
        assert_boxes_close(gb[n].cpu().numpy(), wb)


# ------------------------------------------------------------ Matrix NMS
@pytest.mark.parametrize("M,H,W", [(150, 50, 84), (500, 200, 336)])
def test_matrix_nms_vs_oracle(dev, M, H, W):
    """(500, 200, 336): the C5 geometry -- TOPK_CANDIDATES_TEST = 500 masks of
    the 1333x800 SOLOv2 mask features."""
    rng = np.random.default_rng(51)
    masks = (rng.uniform(size=(M, H, W)) > 0.7).astype(F32)
    for i in range(0, M, 3):  # overlapping pairs
        masks[i + 1] = np.maximum(masks[i], masks[i + 1] * (rng.uniform() > 0.5))
    classes = rng.integers(0, 4, size=M)
    scores = np.sort(rng.uniform(size=M).astype(F32))[::-1].copy()
    for kern in ("gaussian", "linear"):
        want = oracle.matrix_nms(masks, classes, scores, kernel=kern, sigma=2.0)
        got = ops().matrix_nms_scores(torch.from_numpy(masks).to(dev), torch.from_numpy(classes).to(dev),
                                      torch.from_numpy(scores).to(dev), kernel=kern, sigma=2.0)
        g = got.cpu().numpy()
        fin = np.isfinite(want)
        # the finite decays (the linear kernel divides by 1 - comp, which is 0
        # for the duplicated masks: those columns are +inf on both sides)
        np.testing.assert_allclose(g[fin], want[fin], rtol=1e-5, atol=1e-6)
        np.testing.assert_array_equal(g[~fin], want[~fin])
        assert fin.sum() > M // 2


# ------------------------------------------------------------------ conv
@pytest.mark.parametrize("shape", [
    (2, 20, 24, 256, 256, 1, 1, 0),
    (2, 25, 42, 256, 256, 3, 1, 1),
    (1, 17, 9, 64, 96, 3, 2, 1),
    (3, 14, 14, 256, 80, 1, 1, 0),
    (1, 33, 35, 2048, 256, 1, 1, 0),
])
def test_conv2d_mfma_vs_torch_fp32(dev, shape):
    N, H, W, Cin, Cout, k, stride, pad = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(N, H, W, Cin, generator=g)
    w = torch.randn(k, k, Cin, Cout, generator=g) / math.sqrt(k * k * Cin)
    b = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(3, 2, 0, 1).double(),
                                     b.double(), stride=stride, padding=pad).permute(0, 2, 3, 1)
    wp = ops().pack_conv_weights(w.to(dev))
    for relu in (False, True):
        y = ops().conv2d_nhwc(x.to(dev), wp, b.to(dev), stride, (pad, pad), relu)
        want = torch.relu(ref) if relu else ref
        np.testing.assert_allclose(y.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("shape", [
    (2, 20, 24, 256, 256, 1, 1, 0),
    (2, 25, 42, 256, 256, 3, 1, 1),
    (1, 17, 9, 64, 96, 3, 2, 1),
    (3, 14, 14, 256, 80, 1, 1, 0),
    (1, 33, 35, 2048, 256, 1, 1, 0),   # split-K
    (2, 30, 40, 36, 64, 3, 1, 1),      # Cin % 32 != 0 (ragged k-chunk)
    (2, 9, 13, 128, 12, 1, 1, 0),      # Cout 12 (128x32 tile)
])
def test_conv2d_split_bf16_products_are_f32_class(dev, shape):
    """math_mode="split": the f32 operands split exactly into 3 bf16 terms, 6
    bf16 MFMA products (csrc/conv_mfma.hip).  Bar: the same 1e-4 as the native
    f32 path vs float64, and an error no larger than 4x the native f32 MFMA
    path's own (which differs from float64 by summation order only)."""
    N, H, W, Cin, Cout, k, stride, pad = shape
    g = torch.Generator().manual_seed(11 + sum(shape))
    x = torch.randn(N, H, W, Cin, generator=g)
    w = torch.randn(k, k, Cin, Cout, generator=g) / math.sqrt(k * k * Cin)
    b = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(3, 2, 0, 1).double(),
                                     b.double(), stride=stride, padding=pad).permute(0, 2, 3, 1)
    res = torch.randn(ref.shape, generator=g).float()
    wp = ops().pack_conv_weights(w.to(dev))
    for fused in (False, True):
        kw = dict(relu=True, residual=res.to(dev), relu_after_add=True) if fused else {}
        want = torch.relu(ref + res.double()) if fused else ref
        ys = ops().conv2d_nhwc(x.to(dev), wp, b.to(dev), stride, (pad, pad), math_mode="split", **kw)
        yf = ops().conv2d_nhwc(x.to(dev), wp, b.to(dev), stride, (pad, pad), math_mode="f32", **kw)
        ys2 = ops().conv2d_nhwc(x.to(dev), wp, b.to(dev), stride, (pad, pad), math_mode="split", **kw)
        assert torch.equal(ys, ys2)  # deterministic
        np.testing.assert_allclose(ys.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)
        es = float((ys.cpu().double() - want).abs().max())
        ef = float((yf.cpu().double() - want).abs().max())
        assert es <= 4 * ef + 1e-6, (es, ef)


@pytest.mark.parametrize("shape,form", [
    ((2, 40, 52, 64, 256), "r"), ((2, 40, 52, 64, 256), "plain"), ((1, 37, 41, 64, 96), "g"),
    ((2, 33, 40, 128, 512), "gr"), ((2, 33, 40, 128, 128), "plain"), ((1, 29, 31, 128, 192), "r"),
    ((2, 20, 24, 256, 1024), "gr"), ((2, 20, 24, 256, 256), "g"), ((1, 21, 23, 256, 64), "plain"),
    # K = 256 at >= 32 k pixels into 64 / 512 channels: the stream kernel's
    # K = 256 variant ON BY DEFAULT (stream1x1_variant: stream256_shape), whose
    # tiled fallback keeps its tail tiles' K whole -- the shapes above stay
    # under 32 k pixels, where both arms run the tiled kernel
    ((2, 128, 160, 256, 64), "r"), ((2, 128, 160, 256, 64), "g"),
    ((2, 128, 160, 256, 64), "plain"), ((2, 128, 160, 256, 512), "r"),
])
def test_conv1x1_stream_kernel_matches_tiled_and_float64(dev, shape, form):
    """conv1x1_stream_kernel (r5, tuning "conv_stream": the streaming short-K
    1x1 for the memory-bound stride-1 1x1s; weights resident in LDS, pixels
    as the MFMA B operand, float4 epilogue) against float64 (the split
    conv's 1e-4 bar) and against the tiled split kernel on the same launch
    (the same K order and per-accumulator product sequence: equal to the
    tiled kernel's result); ragged pixel strips, Cout not a multiple of the
    slice width, and every epilogue form (bias, residual + ReLU after, ReLU
    gate, gate + residual)."""
    N, H, W, Cin, Cout = shape
    g = torch.Generator().manual_seed(5 + sum(shape))
    x = torch.randn(N, H, W, Cin, generator=g)
    w = torch.randn(1, 1, Cin, Cout, generator=g) / math.sqrt(Cin)
    b = torch.randn(Cout, generator=g) * 0.1
    res = torch.randn(N, H, W, Cout, generator=g) if "r" in form else None
    gate = torch.randn(N, H, W, Cout, generator=g) if "g" in form else None
    ref = torch.einsum("nhwc,cd->nhwd", x.double(), w[0, 0].double()) + b.double()
    if form == "r":
        ref = torch.relu(ref + res.double())
    elif form == "gr":
        ref = torch.where(gate > 0, ref + res.double(), torch.zeros_like(ref))
    elif form == "g":
        ref = torch.where(gate > 0, ref, torch.zeros_like(ref))
    kw = dict(residual=None if res is None else res.to(dev),
              relu_gate=None if gate is None else gate.to(dev),
              relu_after_add=form == "r", relu=form == "r")
    wp = ops().pack_conv_weights(w.to(dev))
    outs = {}
    old = ops().get_tuning("conv_stream")
    try:
        for v in (0, 1):
            ops().set_tuning("conv_stream", v)
            outs[v] = ops().conv2d_nhwc(x.to(dev), wp, b.to(dev), 1, (0, 0), math_mode="split",
                                        **kw).cpu()
    finally:
        ops().set_tuning("conv_stream", old)
    np.testing.assert_allclose(outs[1].double().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    assert torch.equal(outs[0], outs[1])
    if Cin == 256 and N * H * W >= 32768:
        # and with the stream kernel forced (tuning < 0: every eligible launch
        # of >= -value pixels), whatever the default selection rule says
        try:
            ops().set_tuning("conv_stream", -32768)
            forced = ops().conv2d_nhwc(x.to(dev), wp, b.to(dev), 1, (0, 0), math_mode="split",
                                       **kw).cpu()
        finally:
            ops().set_tuning("conv_stream", old)
        assert torch.equal(forced, outs[0])


def test_split_bf16x3_is_exact(dev):
    """h + m + l == x bit for bit (evaluated in float64), each term a bf16.
    Exact wherever the residuals stay normal f32 (|x| >= 2^-110 or so); below
    that the GPU flushes the denormal residual, an error < 2^-126 absolute."""
    g = torch.Generator().manual_seed(9)
    x = torch.cat([torch.randn(4096, generator=g) * 10.0 ** torch.randint(-20, 20, (4096,), generator=g),
                   torch.tensor([0.0, -0.0, 1.0, -1.5, 3.4e38, 2.0 ** -100, 65504.0, 1 + 2.0 ** -23])])
    x3 = ops().split_bf16x3(x.to(dev)).cpu()
    parts = [(x3[i].to(torch.int32) << 16).view(torch.float32).double() for i in range(3)]
    assert torch.equal(parts[0] + parts[1] + parts[2], x.double())


def test_conv2d_split_bf16_exact_on_bf16_representable_integers(dev):
    """Small integers are exact in every term (h = x, m = l = 0) and their
    products and sums are exact in f32: the split path must be bit-exact."""
    g = torch.Generator().manual_seed(5)
    x = torch.randint(-8, 9, (2, 12, 14, 64), generator=g).float()
    w = torch.randint(-4, 5, (3, 3, 64, 96), generator=g).float()
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(3, 2, 0, 1).double(),
                                     padding=1).permute(0, 2, 3, 1)
    y = ops().conv2d_nhwc(x.to(dev), ops().pack_conv_weights(w.to(dev)), None, 1, (1, 1),
                          math_mode="split")
    assert torch.equal(y.cpu().double(), ref)
    # and a value with all three terms non-zero: 1 + 2^-9 + 2^-17 (exact split)
    v = 1.0 + 2.0 ** -9 + 2.0 ** -17
    xo = torch.full((1, 1, 1, 32), v)
    wo = torch.zeros(1, 1, 32, 4)
    wo[0, 0, 0, 0] = 1.0
    wo[0, 0, 0, 1] = v
    y = ops().conv2d_nhwc(xo.to(dev), ops().pack_conv_weights(wo.to(dev)), None, 1, (0, 0),
                          math_mode="split").cpu()
    assert float(y[0, 0, 0, 0]) == np.float32(v)
    assert abs(float(y[0, 0, 0, 1]) - v * v) <= 2.0 ** -22


def test_conv2d_fused_topdown_add(dev):
    """FPN merge prev = lateral(x) + up2(prev_top) fused in the epilogue."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 50, 84, 1024, generator=g)
    w = torch.randn(1, 1, 1024, 256, generator=g) / 32
    b = torch.randn(256, generator=g)
    top = torch.randn(2, 25, 42, 256, generator=g)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(3, 2, 0, 1).double(),
                                     b.double()).permute(0, 2, 3, 1)
    ref = ref + top.double().repeat_interleave(2, 1).repeat_interleave(2, 2)
    y = ops().conv2d_nhwc(x.to(dev), ops().pack_conv_weights(w.to(dev)), b.to(dev),
                          topdown=top.to(dev))
    np.testing.assert_allclose(y.cpu().double().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("shape", [(2, 25, 42, 256, 256, 3, 1, 1), (2, 50, 84, 1024, 64, 1, 2, 0),
                                   (1, 7, 11, 2048, 15, 1, 1, 0)])
def test_conv2d_residual_relu_after_and_split_k(dev, shape):
    """relu(conv + bias + residual) fused (bottleneck epilogue); small-M shapes
    take the split-K path with the fixed-order reduction (deterministic)."""
    N, H, W, Cin, Cout, k, stride, pad = shape
    g = torch.Generator().manual_seed(7 + sum(shape))
    x = torch.randn(N, H, W, Cin, generator=g)
    w = torch.randn(k, k, Cin, Cout, generator=g) / math.sqrt(k * k * Cin)
    b = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(3, 2, 0, 1).double(),
                                     b.double(), stride=stride, padding=pad).permute(0, 2, 3, 1)
    res = torch.randn(ref.shape, generator=g).float()
    want = torch.relu(ref + res.double())
    wp = ops().pack_conv_weights(w.to(dev))
    y1 = ops().conv2d_nhwc(x.to(dev), wp, b.to(dev), stride, (pad, pad), relu=True,
                           residual=res.to(dev), relu_after_add=True)
    y2 = ops().conv2d_nhwc(x.to(dev), wp, b.to(dev), stride, (pad, pad), relu=True,
                           residual=res.to(dev), relu_after_add=True)
    assert torch.equal(y1, y2)
    np.testing.assert_allclose(y1.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("conf", [
    # N, H, W, Cin, Cout, k, stride, relu, topdown, residual
    (2, 25, 42, 256, 256, 3, 1, True, False, False),   # FPN/RPN/mask 3x3: MFMA dgrad
    (2, 50, 84, 512, 256, 1, 1, False, True, False),   # FPN lateral + top-down
    (2, 50, 84, 1024, 256, 1, 1, False, False, True),  # bottleneck conv3 + residual
    (2, 50, 84, 512, 1024, 1, 2, False, False, False), # strided shortcut: GEMM + scatter
    (1, 13, 21, 256, 3, 1, 1, False, False, False),    # objectness 1x1: Cout=3 dgrad fallback
    (1, 17, 9, 64, 96, 3, 2, True, False, False),      # 3x3 stride 2: MIOpen fallback
])
def test_conv_mfma_autograd_matches_torch(dev, conf):
    """Gradients of the MFMA conv layer (x, w, b, top-down, residual) vs
    autograd of the fp64 torch reference."""
    from detectron2_tensorflow_amd.layers.convolutional import _ConvMFMAFn, same_pads
    N, H, W, Cin, Cout, k, stride, relu, td, res = conf
    g = torch.Generator().manual_seed(sum(conf[:7]))
    x = torch.randn(N, H, W, Cin, generator=g)
    w = torch.randn(k, k, Cin, Cout, generator=g) / math.sqrt(k * k * Cin)
    b = torch.randn(Cout, generator=g)
    pads = same_pads(k)
    OH = (H + sum(pads) - k) // stride + 1
    OW = (W + sum(pads) - k) // stride + 1
    top = torch.randn(N, (OH + 1) // 2, (OW + 1) // 2, Cout, generator=g) if td else None
    resid = torch.randn(N, OH, OW, Cout, generator=g) if res else None
    gy = torch.randn(N, OH, OW, Cout, generator=g)

    def ref_fn(x, w, b, top, resid):
        xp = torch.nn.functional.pad(x, (0, 0, pads[0], pads[1], pads[0], pads[1]))
        y = torch.nn.functional.conv2d(xp.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), b,
                                       stride=stride).permute(0, 2, 3, 1)
        if top is not None:
            y = y + top.repeat_interleave(2, 1).repeat_interleave(2, 2)[:, :OH, :OW]
        if resid is not None:
            y = y + resid
        return torch.relu(y) if relu else y

    leaves = [t.double().requires_grad_(True) if t is not None else None
              for t in (x, w, b, top, resid)]
    ref_fn(*leaves).backward(gy.double())
    dl = [t.to(dev).requires_grad_(True) if t is not None else None for t in (x, w, b, top, resid)]
    wp = ops().pack_conv_weights(dl[1].detach())
    y = _ConvMFMAFn.apply(dl[0], dl[1], dl[2], wp, stride, pads, relu, dl[3], dl[4],
                          relu and (td or res))
    y.backward(gy.to(dev))
    for name, a, r in zip("x w b top res".split(), dl, leaves):
        if a is None:
            continue
        np.testing.assert_allclose(a.grad.cpu().double().numpy(), r.grad.numpy(), rtol=1e-4,
                                   atol=2e-4 * max(1.0, float(r.grad.abs().max())), err_msg=name)


@pytest.mark.parametrize("mode", ["f32", "split"])
@pytest.mark.parametrize("conf", [(2, 40, 52, 256, 256, 3, 1), (2, 30, 41, 64, 96, 3, 2),
                                  (2, 200, 168, 256, 64, 1, 1), (1, 50, 84, 512, 1024, 1, 2),
                                  (3, 14, 14, 36, 20, 3, 1)])
def test_conv2d_wgrad_kernel_with_bias(dev, conf, mode):
    """d2mi_conv2d_wgrad_ex (and its fused bias gradient), f32 and split
    products, vs float64 torch."""
    N, H, W, Cin, Cout, k, s = conf
    g = torch.Generator().manual_seed(sum(conf))
    p = (k - 1) // 2
    x = torch.randn(N, H, W, Cin, generator=g)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(N, OH, OW, Cout, generator=g)
    want = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).double(), (Cout, Cin, k, k),
                                       dy.permute(0, 3, 1, 2).double(), s, p).permute(2, 3, 1, 0)
    dw, db = ops().conv2d_wgrad(x.to(dev), dy.to(dev), k, s, (p, p), with_bias=True,
                                math_mode=mode)
    scale = float(want.abs().max())
    np.testing.assert_allclose(dw.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=2e-5 * scale)
    np.testing.assert_allclose(db.cpu().double().numpy(), dy.double().sum((0, 1, 2)).numpy(),
                               rtol=1e-4, atol=1e-3)
    dw2, db2 = ops().conv2d_wgrad(x.to(dev), dy.to(dev), k, s, (p, p), with_bias=True,
                                  math_mode=mode)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("conf", [(2, 200, 336, 256, 256, 1, 1), (2, 100, 168, 512, 1024, 1, 2),
                                  (2, 40, 52, 256, 256, 3, 1)])
def test_conv2d_wgrad_ws_1x1_vs_float64(dev, conf):
    """The warp-specialised wgrad kernel on the large 1x1 convs too (tuning
    "wgrad_ws1", >= 6 GFLOP): vs float64, bias gradient included,
    deterministic."""
    N, H, W, Cin, Cout, k, s = conf
    g = torch.Generator().manual_seed(7 + sum(conf))
    p = (k - 1) // 2
    x = torch.randn(N, H, W, Cin, generator=g)
    OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = torch.randn(N, OH, OW, Cout, generator=g)
    want = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).double(), (Cout, Cin, k, k),
                                       dy.permute(0, 3, 1, 2).double(), s, p).permute(2, 3, 1, 0)
    run = lambda: ops().conv2d_wgrad(x.to(dev), dy.to(dev), k, s, (p, p), with_bias=True,
                                     math_mode="split")
    ops().set_tuning("wgrad_ws1", 6)  # (the default: >= 6 GFLOP)
    dw, db = run()
    dw2, db2 = run()
    scale = float(want.abs().max())
    np.testing.assert_allclose(dw.cpu().double().numpy(), want.numpy(), rtol=1e-4, atol=2e-5 * scale)
    np.testing.assert_allclose(db.cpu().double().numpy(), dy.double().sum((0, 1, 2)).numpy(),
                               rtol=1e-4, atol=1e-3)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("with_bias", [False, True])
def test_fold_frozen_bn_forward_backward(dev, with_bias):
    g = torch.Generator().manual_seed(5)
    KH, Cin, Cout = 3, 64, 128
    w = torch.randn(KH, KH, Cin, Cout, generator=g)
    bias = torch.randn(Cout, generator=g) if with_bias else None
    gamma, beta = torch.rand(Cout, generator=g) + 0.5, torch.randn(Cout, generator=g)
    mean, var = torch.randn(Cout, generator=g), torch.rand(Cout, generator=g) + 0.1
    gw_eff, gb_eff = torch.randn(KH, KH, Cin, Cout, generator=g), torch.randn(Cout, generator=g)

    def ref(w, bias, gamma, beta):
        scale = gamma / torch.sqrt(var.double() + 1e-5)
        b = beta - mean.double() * scale + (bias * scale if bias is not None else 0)
        return w * scale, b

    lv = [t.double().requires_grad_(True) if t is not None else None for t in (w, bias, gamma, beta)]
    rw, rb = ref(*lv)
    (rw * gw_eff.double()).sum().add((rb * gb_eff.double()).sum()).backward()
    dv = [t.to(dev).requires_grad_(True) if t is not None else None for t in (w, bias, gamma, beta)]
    we, be, packed = ops().fold_frozen_bn(dv[0], dv[1], dv[2], dv[3], mean.to(dev), var.to(dev),
                                          1e-5, want_packed=True)
    np.testing.assert_allclose(we.detach().cpu().double().numpy(), rw.detach().numpy(), rtol=1e-5,
                               atol=1e-5)
    np.testing.assert_allclose(be.detach().cpu().double().numpy(), rb.detach().numpy(), rtol=1e-5,
                               atol=1e-5)
    assert torch.equal(packed, ops().pack_conv_weights(we.detach()))
    ((we * gw_eff.to(dev)).sum() + (be * gb_eff.to(dev)).sum()).backward()
    for name, a, r in zip(["w", "bias", "gamma", "beta"], dv, lv):
        if a is None:
            continue
        np.testing.assert_allclose(a.grad.cpu().double().numpy(), r.grad.numpy(), rtol=1e-4,
                                   atol=1e-3, err_msg=name)


@pytest.mark.parametrize("frozen_affine", [False, True])
def test_fold_frozen_bn_many_bit_identical_to_per_conv(dev, frozen_affine):
    """d2mi_fold_frozen_bn_many / _bwd_many (one table-driven launch for every
    conv) give the per-conv fold's w_eff, b_eff, packed and all four
    gradients bit for bit -- mixed shapes (ci / co tails, 7x7 stem, Cout 2048),
    entries with and without bias / packed / a gradient; frozen_affine: gamma
    and beta constants (FrozenBN, the training step's case: the batched
    backward then skips the gamma sums and the read of w, float4 rows)."""
    g = torch.Generator().manual_seed(11)
    shapes = [(7, 7, 3, 64), (1, 1, 64, 256), (3, 3, 60, 36), (1, 1, 1024, 2048), (3, 3, 128, 128),
              (1, 1, 256, 16)]
    entries, grads = [], []
    for i, (kh, kw, ci, co) in enumerate(shapes):
        r = lambda *s: torch.randn(*s, generator=g)
        ts = [r(kh, kw, ci, co), r(co) if i % 2 else None, torch.rand(co, generator=g) + 0.5,
              r(co), r(co), torch.rand(co, generator=g) + 0.1]
        entries.append((ts, 1e-5 if i % 3 else 1e-3, i != 3))
        grads.append((r(kh, kw, ci, co), r(co) if i != 4 else None))

    def run(batched):
        trainable = (0, 1) if frozen_affine else (0, 1, 2, 3)
        leaves = [[t.to(dev).requires_grad_(k in trainable) if t is not None else None
                   for k, t in enumerate(ts)] for ts, _, _ in entries]
        if batched:
            outs = ops().fold_frozen_bn_many([(*lv, eps, pk) for lv, (_, eps, pk)
                                              in zip(leaves, entries)])
        else:
            outs = [ops().fold_frozen_bn(*lv, eps, pk) for lv, (_, eps, pk) in zip(leaves, entries)]
        ys, gs = [], []
        for (we, be, _), (gw, gb) in zip(outs, grads):
            ys.append(we)
            gs.append(gw.to(dev))
            if gb is not None:  # else b_eff gets no gradient at all
                ys.append(be)
                gs.append(gb.to(dev))
        torch.autograd.backward(ys, gs)
        return outs, leaves

    a, la = run(True)
    b, lb = run(False)
    for (wa, ba, pa), (wb, bb, pb) in zip(a, b):
        assert torch.equal(wa, wb) and torch.equal(ba, bb)
        assert (pa is None) == (pb is None) and (pa is None or torch.equal(pa, pb))
    for xa, xb in zip(la, lb):
        for ta, tb in zip(xa[:4], xb[:4]):
            if ta is not None and ta.requires_grad:
                assert torch.equal(ta.grad, tb.grad)


@pytest.mark.parametrize("H,W,fixed", [(96, 128, False), (75, 101, False), (64, 64, True)])
def test_paste_masks_bit_exact(dev, H, W, fixed):
    """d2mi_paste_masks vs the oracle (crop_and_resize of the reverse box +
    tf.greater): uint8 masks bit-exact, including boxes hanging off the canvas,
    sub-pixel boxes, invalid slots and the 'fixed' per-box scale."""
    rng = np.random.default_rng(H * W)
    D = 37
    m = rng.random((D, 28, 28)).astype(F32)
    y1 = rng.uniform(-20, H, D)
    x1 = rng.uniform(-20, W, D)
    b = np.stack([y1, x1, y1 + rng.uniform(0.3, H, D), x1 + rng.uniform(0.3, W, D)], 1).astype(F32)
    valid = rng.random(D) < 0.8
    yx = rng.uniform(0.5, 2.0, (D, 2)).astype(F32) if fixed else None
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    got = ops().paste_masks(t(m), t(b), (H, W), valid=t(valid), yx_scale=t(yx))
    want = oracle.paste_masks(m, b, (H, W), valid=valid, yx_scale=yx)
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    assert want.sum() > 0
    empty = ops().paste_masks(t(m[:0]), t(b[:0]), (H, W))
    assert tuple(empty.shape) == (0, H, W)


@pytest.mark.parametrize("shape", [(3, 3, 64, 64), (1, 1, 256, 16), (1, 1, 1024, 80),
                                   (3, 3, 60, 36), (1, 1, 2048, 512), (7, 7, 3, 64)])
def test_weight_pack_and_frozen_bn_fold_layouts(dev, shape):
    """pack_conv_weights: HWIO -> [KH, KW, Cout, Cin] bit-exact (tiled path for
    Cin % 64 == 0, element path otherwise); the FrozenBN fold writes
    w_eff = w * gamma / sqrt(var + eps) and its packed copy consistently."""
    g = torch.Generator().manual_seed(sum(shape))
    w = torch.randn(shape, generator=g).to(dev)
    np.testing.assert_array_equal(ops().pack_conv_weights(w).cpu().numpy(),
                                  w.permute(0, 1, 3, 2).cpu().numpy())
    Cout = shape[3]
    gamma, beta = torch.rand(Cout, generator=g) + 0.5, torch.randn(Cout, generator=g)
    mean, var = torch.randn(Cout, generator=g), torch.rand(Cout, generator=g) + 0.1
    t = lambda a: a.to(dev)
    with torch.no_grad():
        w_eff, b_eff, packed = ops().fold_frozen_bn(w, None, t(gamma), t(beta), t(mean), t(var),
                                                    1e-5, True)
    scale = gamma / torch.sqrt(var + 1e-5)
    torch.testing.assert_close(w_eff.cpu(), w.cpu() * scale, rtol=1e-6, atol=0)
    torch.testing.assert_close(b_eff.cpu(), beta - mean * scale, rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(packed.cpu().numpy(), w_eff.permute(0, 1, 3, 2).cpu().numpy())


def test_column_sum_and_linear_mfma_match_float64(dev):
    """Bias-gradient column sums (d2mi_column_sum) and the long-K Linear on the
    split-product MFMA kernels (fwd, dgrad, wgrad + bias grad) vs float64."""
    from detectron2_tensorflow_amd.layers import Linear
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 50, 84, 1024, generator=g)
    got = ops().column_sum(x.to(dev)).cpu().double()
    torch.testing.assert_close(got, x.double().sum((0, 1, 2)), rtol=1e-5, atol=1e-4)
    lin = Linear(4352, 132).to(dev)
    with torch.no_grad():
        lin.bias.normal_()
    xi = torch.randn(300, 4352, generator=g).to(dev).requires_grad_(True)
    y = lin(xi)
    gy = torch.randn(y.shape, generator=g).to(dev)
    y.backward(gy)
    xd, wd, gd = xi.detach().double(), lin.weights.detach().double(), gy.double()
    torch.testing.assert_close(y.double(), xd @ wd + lin.bias.detach().double(), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(xi.grad.double(), gd @ wd.t(), rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(lin.weights.grad.double(), xd.t() @ gd, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(lin.bias.grad.double(), gd.sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("declared", [True, False])
def test_relu_gate_fused_into_consumer_dgrad(dev, declared):
    """conv(relu) -> conv(relu) -> conv chains: a consumer declared as the sole
    consumer of a fused-ReLU output applies that ReLU's backward in its own
    dgrad epilogue (kMaskByResidual) and the producer skips its own; without
    the declaration nothing is fused.  Gradients match float64 autograd."""
    from detectron2_tensorflow_amd.layers.convolutional import _ConvMFMAFn
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, 12, 15, 64, generator=g)
    ws = [torch.randn(3, 3, 64, 64, generator=g) / 24 for _ in range(3)]
    bs = [torch.randn(64, generator=g) * 0.1 for _ in range(3)]
    gy = torch.randn(2, 12, 15, 64, generator=g)

    def ref(h, ws, bs):
        for i, (w, b) in enumerate(zip(ws, bs)):
            h = torch.nn.functional.conv2d(h.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), b,
                                           padding=1).permute(0, 2, 3, 1)
            if i < 2:
                h = torch.relu(h)
        return h

    lx = [t.double().requires_grad_(True) for t in [x] + ws + bs]
    ref(lx[0], lx[1:4], lx[4:7]).backward(gy.double())
    dx = [t.to(dev).requires_grad_(True) for t in [x] + ws + bs]
    h = dx[0]
    outs = []
    for i in range(3):
        w, b = dx[1 + i], dx[4 + i]
        h = _ConvMFMAFn.apply(h, w, b, ops().pack_conv_weights(w.detach()), 1, (1, 1), i < 2,
                              None, None, False, declared and i > 0)
        outs.append(h)
    h.backward(gy.to(dev))
    assert outs[0]._d2mi_relu_info["masked"] is declared
    assert outs[1]._d2mi_relu_info["masked"] is declared
    for name, a, r in zip(["x", "w0", "w1", "w2", "b0", "b1", "b2"], dx, lx):
        np.testing.assert_allclose(a.grad.cpu().double().numpy(), r.grad.numpy(), rtol=1e-4,
                                   atol=2e-4 * max(1.0, float(r.grad.abs().max())), err_msg=name)


@pytest.mark.parametrize("C", [256])
@pytest.mark.parametrize("epi", ["relu", "residual", "topdown"])
def test_conv2d_tail_split_matches_float64(dev, epi, C):
    """Grids a little over one round of resident workgroups (C=256: 2x100x168
    -> 263 x 2 = 526 tiles of 128x128) run their last pixel-row blocks as a
    split-K tail launch with a fixed-order reduce; every epilogue form stays
    within the f32-class bound of float64."""
    g = torch.Generator().manual_seed(3)
    N, H, W = 2, 100, 168
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(3, 3, C, C, generator=g) / math.sqrt(9 * C)
    b = torch.randn(C, generator=g)
    res = torch.randn(N, H, W, C, generator=g) if epi == "residual" else None
    top = torch.randn(N, H // 2, W // 2, C, generator=g) if epi == "topdown" else None
    ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2),
                                     w.double().permute(3, 2, 0, 1), b.double(),
                                     padding=1).permute(0, 2, 3, 1)
    if res is not None:
        ref = ref + res.double()
    if top is not None:
        ref = ref + top.double().repeat_interleave(2, 1).repeat_interleave(2, 2)
    if epi == "relu":
        ref = ref.clamp(min=0)
    t = lambda a: None if a is None else a.to(dev)
    y = ops().conv2d_nhwc(t(x), ops().pack_conv_weights(t(w)), t(b), 1, (1, 1),
                          relu=epi == "relu", residual=t(res), topdown=t(top))
    np.testing.assert_allclose(y.cpu().double().numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)
    # the tail rows (the last 14 tiles) are really there
    assert torch.isfinite(y[-1, -1]).all() and float(y[-1, -1].abs().sum()) > 0


@pytest.mark.parametrize("shape", [(2, 50, 84, 256, 64, 1), (2, 25, 42, 512, 2048, 1),
                                   (2, 12, 15, 64, 64, 3), (1, 100, 168, 128, 512, 1)])
def test_gated_conv_adds_residual_then_masks(dev, shape):
    """d2mi_conv2d_nhwc_gated: y = gate > 0 ? conv + residual : 0 equals the
    ungated conv-with-residual masked afterwards, bit for bit -- whole tiles,
    split-K (small M) and the tail split, flipped taps for the 3x3 dgrad."""
    N, H, W, Cin, Cout, k = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(N, H, W, Cin, generator=g).to(dev)
    w = (torch.randn(k, k, Cout, Cin, generator=g) / Cin ** 0.5).to(dev)
    res = torch.randn(N, H, W, Cout, generator=g).to(dev)
    gate = torch.relu(torch.randn(N, H, W, Cout, generator=g)).to(dev)
    p = (k // 2, k // 2)
    for flip in ([False, True] if k > 1 else [False]):
        want = ops().conv2d_nhwc(x, w, None, 1, p, residual=res, flip_taps=flip)
        want = torch.where(gate > 0, want, torch.zeros_like(want))
        got = ops().conv2d_nhwc(x, w, None, 1, p, residual=res, relu_gate=gate, flip_taps=flip)
        assert torch.equal(got, want)
        plain = ops().conv2d_nhwc(x, w, None, 1, p, relu_gate=gate, flip_taps=flip)
        ref = ops().conv2d_nhwc(x, w, None, 1, p, flip_taps=flip)
        assert torch.equal(plain, torch.where(gate > 0, ref, torch.zeros_like(ref)))


@pytest.mark.parametrize("stride", [1, 2])
def test_bottleneck_residual_gradient_handoff_is_exact(dev, stride):
    """A res3-like stage (block 1's conv1 / projection shortcut meet in one
    dgrad epilogue; blocks 2..3 hand their identity-shortcut gradient to
    conv1's gated dgrad) gives exactly the gradients of the same stage with the
    hand-offs off (autograd add + ReLU backward; the latter is checked against
    float64 autograd by test_relu_gate_fused_into_consumer_dgrad)."""
    from detectron2_tensorflow_amd.modeling.backbone.resnet import BottleneckBlock, Stage
    torch.manual_seed(3)
    st = Stage(BottleneckBlock, {"in_channels": 64, "out_channels": 128,
                                 "bottleneck_channels": 32, "stride_in_1x1": True}, 3, stride,
               scope="res_t").to(dev)
    assert [b.grad_handoff for b in st.blocks] == [False, True, True]
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 20, 24, 64, generator=g).to(dev)
    gy = torch.randn(2, 20 // stride, 24 // stride, 128, generator=g).to(dev)
    res = {}
    for handoff in (True, False):
        for b in st.blocks[1:]:
            b.grad_handoff = handoff
        st.blocks[0].grad_pair = handoff
        st.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        y = st(xi)
        y.backward(gy)
        res[handoff] = (y.detach(), xi.grad, {n: p.grad.clone() for n, p in st.named_parameters()})
    ya, gxa, gpa = res[True]
    yb, gxb, gpb = res[False]
    assert torch.equal(ya, yb) and torch.equal(gxa, gxb)
    assert gpa.keys() == gpb.keys() and gpa
    for n in gpa:
        assert torch.equal(gpa[n], gpb[n]), n


@pytest.mark.parametrize("shape", [(2, 25, 42, 256), (1, 7, 5, 8), (2, 200, 336, 16)])
def test_upsample2x_grad_and_stride_scatter(dev, shape):
    """d2mi_upsample2x_grad equals the 2x2 sum-pool of the zero-padded gradient
    (odd maps included); d2mi_stride_scatter equals zeros + strided copy (+ add)."""
    g = torch.Generator().manual_seed(sum(shape))
    N, H, W, C = shape
    gy = torch.randn(N, H, W, C, generator=g)
    want = torch.nn.functional.pad(gy.double(), (0, 0, 0, W % 2, 0, H % 2))
    want = want.reshape(N, (H + 1) // 2, 2, (W + 1) // 2, 2, C).sum((2, 4))
    got = ops().upsample2x_grad(gy.to(dev)).cpu().double()
    np.testing.assert_allclose(got.numpy(), want.numpy(), rtol=1e-6, atol=1e-6)
    for s in (2, 3):
        gs = torch.randn(N, (H - 1) // s + 1, (W - 1) // s + 1, C, generator=g)
        add = torch.randn(N, H, W, C, generator=g)
        ref = torch.zeros(N, H, W, C)
        ref[:, ::s, ::s] = gs
        assert torch.equal(ops().stride_scatter(gs.to(dev), (N, H, W, C), s).cpu(), ref)
        assert torch.equal(ops().stride_scatter(gs.to(dev), (N, H, W, C), s, add.to(dev)).cpu(),
                           ref + add)


def test_stride_scatter_two_adds_and_gate(dev):
    """d2mi_stride_scatter_ex: ((scatter + add) + add2) then the ReLU backward
    of the gate tensor, exactly as torch forms it (threshold_backward)."""
    g = torch.Generator().manual_seed(11)
    N, H, W, C, s = 2, 13, 10, 12, 2
    gs = torch.randn(N, (H - 1) // s + 1, (W - 1) // s + 1, C, generator=g)
    add, add2 = torch.randn(N, H, W, C, generator=g), torch.randn(N, H, W, C, generator=g)
    gate = torch.relu(torch.randn(N, H, W, C, generator=g))
    ref = torch.zeros(N, H, W, C)
    ref[:, ::s, ::s] = gs
    want = torch.ops.aten.threshold_backward((ref + add) + add2, gate, 0.0)
    got = ops().stride_scatter(gs.to(dev), (N, H, W, C), s, add.to(dev), add2.to(dev), gate.to(dev))
    assert torch.equal(got.cpu(), want)
    got = ops().stride_scatter(gs.to(dev), (N, H, W, C), s, gate=gate.to(dev))
    assert torch.equal(got.cpu(), torch.ops.aten.threshold_backward(ref, gate, 0.0))


@pytest.mark.parametrize("lateral_first", [False, True])
def test_stage_output_join_with_fpn_lateral_is_exact(dev, lateral_first):
    """A ReLU output (a stage output) read by the next stage's strided conv1 /
    projection-shortcut pair and by an FPN lateral (with its fused top-down
    add): the three-consumer join (the last backward adds the others'
    gradients and applies the producer's ReLU mask) gives exactly the
    gradients of the autograd formulation (adds + threshold_backward).  The
    lateral created first runs its backward last (autograd runs ready nodes
    by creation order, newest first): both completion orders are exercised."""
    from detectron2_tensorflow_amd.layers import Conv2D
    torch.manual_seed(5)
    prod = Conv2D(64, 128, 3, activation="relu", impl="mfma", scope="prod").to(dev)
    conv1 = Conv2D(128, 32, 1, stride=2, impl="mfma", scope="conv1").to(dev)
    short = Conv2D(128, 256, 1, stride=2, activation=None, impl="mfma", scope="shortcut").to(dev)
    lat = Conv2D(128, 64, 1, activation=None, impl="mfma", scope="lat").to(dev)
    mods = (prod, conv1, short, lat)
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 20, 24, 64, generator=g).to(dev)
    td = torch.randn(2, 10, 12, 64, generator=g).to(dev)
    gh = torch.randn(2, 10, 12, 32, generator=g).to(dev)
    gs = torch.randn(2, 10, 12, 256, generator=g).to(dev)
    gl = torch.randn(2, 20, 24, 64, generator=g).to(dev)
    res = {}
    for join in (True, False):
        for m in mods:
            m.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        c = prod(xi)
        pair = {}
        if lateral_first:
            lo = lat(c, topdown=td, join=pair if join else None)
        sc = short(c, pair_grad=pair)
        h = conv1(c, pair_grad=pair)
        if not lateral_first:
            lo = lat(c, topdown=td, join=pair if join else None)
        torch.autograd.backward([h, sc, lo], [gh, gs, gl])
        if join:
            assert pair.get("last") == ("lateral" if lateral_first else "pair")
            assert not ({"g", "sum", "lat"} & pair.keys())  # nothing left behind
        res[join] = (xi.grad, {n: q.grad.clone() for m in mods for n, q in m.named_parameters()})
    gxa, gpa = res[True]
    gxb, gpb = res[False]
    assert torch.equal(gxa, gxb)
    assert gpa.keys() == gpb.keys() and gpa
    for n in gpa:
        assert torch.equal(gpa[n], gpb[n]), n


@pytest.mark.parametrize("allow_low,per_image", [(True, False), (False, True)])
def test_fused_match_equals_tensor_matcher(dev, allow_low, per_image):
    """d2mi_match_boxes (IoU + Matcher in one pass) gives the tensor
    formulation's matches and labels exactly: crowd and difficult GT, padded
    (invalid) GT, an image without any matchable GT, IoU ties (duplicate GT),
    boxes shared by the batch or per image."""
    from detectron2_tensorflow_amd.modeling.matcher import Matcher, match_boxes
    rng = np.random.default_rng(5 + int(allow_low))
    N, G, P = 3, 9, 5000
    def boxes(k):
        cy, cx = rng.uniform(0, 400, k), rng.uniform(0, 600, k)
        h, w = rng.uniform(4, 200, k), rng.uniform(4, 200, k)
        return np.stack([cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2], -1).astype(F32)
    gt = boxes(N * G).reshape(N, G, 4)
    gt[0, 1] = gt[0, 0]  # a tie
    bx = boxes(N * P).reshape(N, P, 4) if per_image else boxes(P)
    bx[..., :7, :] = gt[0, :7] if not per_image else gt[:, :7]  # exact hits
    valid = rng.random((N, G)) < 0.8
    valid[2] = False
    crowd = rng.random((N, G)) < 0.2
    diff = rng.random((N, G)) < 0.2
    m = Matcher([0.3, 0.7], [0, -1, 1], allow_low_quality_matches=allow_low)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a))
    args = (t(gt), t(valid & ~crowd & ~diff), t(bx))
    want = match_boxes(m, *args, crowd=t(crowd), difficult=t(diff))
    got = match_boxes(m, *[a.to(dev) for a in args], crowd=t(crowd).to(dev),
                      difficult=t(diff).to(dev))
    assert torch.equal(got[0].cpu(), want[0]) and torch.equal(got[1].cpu(), want[1])
    assert (want[1] == 1).any() and (want[1] == -1).any() and (want[1] == 0).any()


def test_match_masks_abi_equals_packed_flags(dev):
    """d2mi_match_boxes_ex (byte masks, crowd / difficult optional; matchable
    = valid and neither crowd nor difficult) == the packed-int32
    d2mi_match_boxes on the same GT, with and without the optional masks."""
    from detectron2_tensorflow_amd.layers import ops
    g = torch.Generator().manual_seed(9)
    N, G, P = 2, 12, 3000
    def boxes(k):
        c = torch.rand(k, 2, generator=g) * 400
        hw = torch.rand(k, 2, generator=g) * 150 + 4
        return torch.cat([c - hw / 2, c + hw / 2], 1)
    gt = boxes(N * G).reshape(N, G, 4).to(dev)
    bx = boxes(P).to(dev)
    valid = (torch.rand(N, G, generator=g) < 0.8).to(dev)
    crowd = (torch.rand(N, G, generator=g) < 0.3).to(dev)
    diff = (torch.rand(N, G, generator=g) < 0.3).to(dev)
    thr, lab = [-math.inf, 0.3, 0.7, math.inf], [0, -1, 1]
    for c, d in ((crowd, diff), (None, diff), (crowd, None), (None, None)):
        m = valid
        if c is not None:
            m = m & ~c
        if d is not None:
            m = m & ~d
        flags = m.to(torch.int32)
        if c is not None:
            flags = flags | (c.to(torch.int32) << 1)
        if d is not None:
            flags = flags | (d.to(torch.int32) << 2)
        kw = dict(crowd_thr=1e-3, difficult_thr=0.3)
        want = ops.match_boxes(gt, flags, bx, thr, lab, True, **kw)
        got = ops.match_boxes_masks(gt, valid, bx, thr, lab, True, crowd=c, difficult=d, **kw)
        assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1])


def test_sampling_smallest_keys_on_hip_topk(dev):
    """subsample_labels' k-smallest selection on the HIP segmented radix select
    equals torch.topk's on the CPU (distinct keys): per-row limits, rows with
    fewer candidates than k, an empty row."""
    from detectron2_tensorflow_amd.modeling.matcher import _smallest
    g = torch.Generator().manual_seed(9)
    N, P, k = 3, 268569, 256
    keys = torch.randperm(N * P, generator=g).reshape(N, P).float() / (N * P)
    mask = torch.rand(N, P, generator=g) < 0.3
    mask[1] = torch.rand(P, generator=g) < 1e-4  # fewer than k candidates
    mask[2] = False
    limit = torch.tensor([[200], [256], [10]])
    want = _smallest(keys, mask, k, limit)
    got = _smallest(keys.to(dev), mask.to(dev), k, limit.to(dev)).cpu()
    assert torch.equal(got, want)
    assert int(want[0].sum()) == 200 and int(want[1].sum()) == int(mask[1].sum())


def test_fused_stem_pool_matches_unfused(dev):
    """The frozen stem's tail (d2mi_stem_pool: relu(+shift), zero pad, 3x3/2
    VALID pool, here after its MIOpen-conv arm) equals conv + ReLU + F.pad +
    max_pool2d bit for bit (the MFMA conv arm: test_stem_conv_mfma_vs_float64
    and test_stem_mfma_conv_matches_miopen_stem)."""
    from detectron2_tensorflow_amd.layers import BatchNorm
    from detectron2_tensorflow_amd.modeling.backbone.resnet import Stem
    from detectron2_tensorflow_amd.utils.arg_scope import arg_scope
    from detectron2_tensorflow_amd.layers import Conv2D
    torch.manual_seed(2)
    with arg_scope([Conv2D], normalizer=BatchNorm, activation="relu", use_bias=False,
                   impl="auto"):
        stem = Stem(3, 64, scope="stem").to(dev)
    with torch.no_grad():
        n = stem.conv1.normalizer_fn
        n.moving_mean.normal_()
        n.moving_variance.uniform_(0.5, 2.0)
    for p in stem.parameters():
        p.requires_grad_(False)
    x = torch.randn(2, 101, 134, 3, device=dev) * 50
    with torch.no_grad():
        assert stem._fused_ok(x)
        stem.MFMA_CONV = False  # the MIOpen arm: the same conv as the unfused path
        got = stem(x)
        stem._fused_ok = lambda x: False
        want = stem(x)
    assert got.shape == want.shape == (2, 26, 34, 64)
    assert torch.equal(got, want)


@pytest.mark.parametrize("merged", [True, False])
def test_roi_align_backward_grad_share_matches_autograd_sum(dev, merged):
    """Two poolings of the same p2..p5 maps (the box 7x7 and mask 14x14 poolers
    of a training step) with grad_share == autograd's sum of two independent
    backwards, bit for bit: merged = ONE backward over both ROI sets
    (d2mi_roi_align_bwd2: one sort on (pixel, set) keys, each set's run summed
    apart, then added); else the first backward writes the maps and the second
    accumulates into them (d2mi_roi_align_bwd_ex accumulate).  Small boxes
    pile > 64 contributions onto single pixels (the split-run path)."""
    import detectron2_tensorflow_amd.layers.ops as O
    O.MERGED_BWD = merged
    try:
        _grad_share_case(dev)
    finally:
        O.MERGED_BWD = True


def _grad_share_case(dev):
    rng = np.random.default_rng(45)
    N, IH, IW, C = 2, 256, 320, 64
    strides = [4, 8, 16, 32]
    scales = [1.0 / s for s in strides]
    feats = [rng.normal(size=(N, IH // s, IW // s, C)).astype(F32) for s in strides]
    b1, b2 = rand_boxes(rng, 400, IH, IW, 2.0, 300.0), rand_boxes(rng, 64, IH, IW, 8.0, 300.0)
    i1 = rng.integers(0, N, size=400).astype(np.int32)
    i2 = rng.integers(0, N, size=64).astype(np.int32)
    g1 = torch.from_numpy(rng.normal(size=(400, 7, 7, C)).astype(F32)).to(dev)
    g2 = torch.from_numpy(rng.normal(size=(64, 14, 14, C)).astype(F32)).to(dev)
    grads = []
    for share in (None, {}):
        xs = [torch.from_numpy(f).to(dev).requires_grad_(True) for f in feats]
        o1 = ops().roi_align(xs, torch.from_numpy(b1).to(dev), torch.from_numpy(i1).to(dev), (7, 7),
                             scales, 0, True, grad_share=share)
        o2 = ops().roi_align(xs, torch.from_numpy(b2).to(dev), torch.from_numpy(i2).to(dev),
                             (14, 14), scales, 0, True, grad_share=share)
        torch.autograd.backward([o1, o2], [g1, g2])
        grads.append([x.grad.clone() for x in xs])
        assert share is None or not share  # the second backward took the maps
    for a, b in zip(*grads):
        assert torch.equal(a, b)


@pytest.mark.parametrize("cout,relu", [(256, True), (720, False), (36, False)])
def test_conv_levels_matches_per_level_convs(dev, cout, relu):
    """d2mi_conv2d_nhwc_levels (one launch over RetinaNet's P3..P7 at 640x640,
    shared weights) == conv2d_nhwc per level: the same per-tile arithmetic,
    summation order differing only where a small level alone would split K;
    and level 0 vs float64.  Cout 720 = the cls_score head (a partial N tile),
    36 = bbox_pred (narrow: f32 MFMA)."""
    from detectron2_tensorflow_amd.layers import ops
    g = torch.Generator(device="cpu").manual_seed(11)
    shapes = [(2, 80, 80), (2, 40, 40), (2, 20, 20), (2, 10, 10), (2, 5, 5)]
    xs = [torch.randn(n, h, w, 256, generator=g).to(dev) for n, h, w in shapes]
    w = (torch.randn(3, 3, 256, cout, generator=g) * 0.02).to(dev)
    b = (torch.randn(cout, generator=g) * 0.1).to(dev)
    wp = ops.pack_conv_weights(w)
    ys = ops.conv2d_nhwc_levels(xs, wp, b, 1, (1, 1), relu=relu)
    ys2 = ops.conv2d_nhwc_levels(xs, wp, b, 1, (1, 1), relu=relu)
    for y, y2 in zip(ys, ys2):
        assert torch.equal(y, y2)
    for x, y in zip(xs, ys):
        ref = ops.conv2d_nhwc(x, wp, b, 1, (1, 1), relu=relu)
        assert y.shape == ref.shape
        torch.testing.assert_close(y, ref, rtol=1e-5, atol=1e-5 * float(ref.abs().max()))
    x64 = xs[0].double().permute(0, 3, 1, 2)
    r64 = torch.nn.functional.conv2d(x64, w.double().permute(3, 2, 0, 1), b.double(), padding=1)
    r64 = r64.permute(0, 2, 3, 1)
    if relu:
        r64 = r64.clamp_min(0)
    torch.testing.assert_close(ys[0].double(), r64, rtol=1e-4, atol=1e-4)


def test_pack_weights_many_and_pack_group(dev):
    """d2mi_conv_pack_weights_many equals d2mi_conv_pack_weights tensor by
    tensor (tiled Cin % 64 == 0 entries batched, > 32 of them split over
    launches; other Cin alone), and a PackGroup repacks every member whose
    parameters changed in one call, leaving the fresh ones untouched."""
    from detectron2_tensorflow_amd.layers import Conv2D
    from detectron2_tensorflow_amd.layers.convolutional import PackGroup
    g = torch.Generator().manual_seed(21)
    shapes = [(3, 3, 256, 256), (1, 1, 512, 256), (1, 1, 24, 16), (3, 3, 64, 100)] * 9
    ws = [torch.randn(*s, generator=g).to(dev) for s in shapes]
    got = ops().pack_conv_weights_many(ws)
    for w, p in zip(ws, got):
        assert torch.equal(p, ops().pack_conv_weights(w))
    convs = [Conv2D(64, 64, 3, impl="mfma", scope=f"c{i}").to(dev) for i in range(3)]
    grp = PackGroup()
    for c in convs:
        c._pack_group = grp
    x = torch.randn(1, 8, 8, 64, generator=g).to(dev)
    for c in convs:
        c(x)
    assert len(grp.members) == 3
    kept = convs[2]._packed
    with torch.no_grad():
        convs[0].weights.add_(1.0)
        convs[1].weights.mul_(0.5)
    calls = []
    real = ops().pack_conv_weights_many
    try:
        ops().pack_conv_weights_many = lambda ws: calls.append(len(ws)) or real(ws)
        for c in convs:
            c(x)
    finally:
        ops().pack_conv_weights_many = real
    assert calls == [2]
    assert convs[2]._packed is kept
    for c in convs:
        assert torch.equal(c._packed, ops().pack_conv_weights(c.weights.detach()))


@pytest.mark.parametrize("shape", [(2, 64, 96), (1, 37, 53), (2, 800, 1344)])
def test_stem_conv_mfma_vs_float64(dev, shape):
    """d2mi_stem_conv (the frozen stem's 7x7 / stride-2 conv, Cin 3 -> 64,
    fix_padding's symmetric pad 3) on the split-bf16 MFMA vs float64, odd
    sizes (partial 128-pixel tiles, bottom / right padding) and the bench
    geometry; then the whole Stem (conv + shift + ReLU + pad + pool) against
    its MIOpen arm."""
    N, H, W = shape
    g = torch.Generator().manual_seed(H + W)
    x = torch.randn(N, H, W, 3, generator=g) * 50.0
    w = torch.randn(7, 7, 3, 64, generator=g) / math.sqrt(147.0)
    y = ops().stem_conv(x.to(dev), ops().stem_conv_weights(w.to(dev)))
    if N * H * W <= 10000:
        ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(),
                                         w.permute(3, 2, 0, 1).double(), stride=2,
                                         padding=3).permute(0, 2, 3, 1)
    else:  # the first 4 output rows of image 0 (input rows 0..9 + the top pad)
        ref = torch.nn.functional.conv2d(x[:1, :10].permute(0, 3, 1, 2).double(),
                                         w.permute(3, 2, 0, 1).double(), stride=2,
                                         padding=3).permute(0, 2, 3, 1)[:, :4]
        y = y[:1, :4]
    scale = float(ref.abs().max())
    np.testing.assert_allclose(y.cpu().double().numpy(), ref.numpy(), rtol=1e-4, atol=1e-5 * scale)


@pytest.mark.parametrize("shape,div,flip", [((2, 37, 45), 32, True), ((1, 29, 30), 0, False),
                                            ((3, 64, 64), 32, True), ((2, 800, 1333), 32, True)])
def test_preprocess_images_bit_exact(dev, shape, div, flip):
    """d2mi_preprocess_images (normalise, BGR flip, zero pad to the size
    divisibility in one launch) vs the reference's three steps in float32 on
    the CPU (rcnn.py:146-157, image_list.py:89-100; the form of
    oracle/cpu_pipeline.py) -- bit-identical, odd sizes (partial float4 rows,
    no pad, pad on both axes) and the bench geometry, and vs torch's own
    GPU launches of the same steps."""
    N, H, W = shape
    g = torch.Generator().manual_seed(H * W + N)
    x = torch.rand(N, H, W, 3, generator=g) * 255.0
    mean = torch.tensor([123.675, 116.28, 103.53])
    std = torch.tensor([58.395, 57.12, 57.375])
    ref = (x - mean) / std
    if flip:
        ref = ref.flip(-1)
    if div:
        ref = torch.nn.functional.pad(ref, (0, 0, 0, (-W) % div, 0, (-H) % div))
    got = ops().preprocess_images(x.to(dev), mean.to(dev), std.to(dev), flip, div)
    assert got.shape == ref.shape
    assert torch.equal(got.cpu(), ref)
    # the GPU torch form the fused op replaces: the same bits
    t = (x.to(dev) - mean.to(dev)) / std.to(dev)
    t = t.flip(-1) if flip else t
    if div:
        t = torch.nn.functional.pad(t, (0, 0, 0, (-W) % div, 0, (-H) % div))
    assert torch.equal(got, t)


def test_stem_mfma_conv_matches_miopen_stem(dev):
    from detectron2_tensorflow_amd.modeling.backbone.resnet import Stem, resnet_arg_scope
    torch.manual_seed(0)
    with resnet_arg_scope(True, "FrozenBN"):
        stem = Stem(3, 64, scope="stem").to(dev)
    norm = stem.conv1.normalizer_fn  # a non-trivial frozen BN fold
    with torch.no_grad():
        for t in (norm.gamma, norm.beta, norm.moving_mean, norm.moving_variance):
            t.uniform_(0.5, 1.5)
    for t in stem.parameters():
        t.requires_grad_(False)
    x = torch.randn(2, 160, 224, 3, device=dev) * 50.0
    with torch.no_grad():
        Stem.MFMA_CONV = True
        a = stem(x)
        Stem.MFMA_CONV = False
        b = stem(x)
        Stem.MFMA_CONV = True
    np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4,
                               atol=1e-5 * float(b.abs().max()))


def test_fused_subsample_counts_order_and_uniformity(dev):
    """d2mi_subsample (the fused subsample_labels): exact counts
    min(num_pos, #pos) / min(num_samples - that, #neg) inside the masks, the
    fg-first index order, determinism per seed, every element drawn with
    probability k / n (binomial bound over 400 seeds), and all kept when they
    fit."""
    g = torch.Generator().manual_seed(3)
    N, P, S, num_pos, bg = 3, 5000, 512, 128, 80
    lab = torch.randint(-1, 81, (N, P), generator=g)
    lab[1] = torch.where(torch.rand(P, generator=g) < 0.995, torch.full((P,), bg), lab[1])
    lab[2, :] = -1
    lab[2, :40] = 3
    lab[2, 40:100] = bg  # fewer than S candidates: everything kept
    lab = lab.to(dev)
    seed = torch.tensor([12345], dtype=torch.int64, device=dev)
    pos, neg, order, valid = ops().subsample(lab, S, num_pos, bg, seed, order_slots=S)
    pos2, neg2 = ops().subsample(lab, S, num_pos, bg, seed)
    assert torch.equal(pos, pos2) and torch.equal(neg, neg2)
    lc = lab.cpu()
    for r in range(N):
        ispos = (lc[r] != -1) & (lc[r] != bg)
        isneg = lc[r] == bg
        p, q = pos[r].cpu(), neg[r].cpu()
        assert not (p & ~ispos).any() and not (q & ~isneg).any()
        kp = min(num_pos, int(ispos.sum()))
        assert int(p.sum()) == kp
        assert int(q.sum()) == min(S - kp, int(isneg.sum()))
        want = torch.cat([torch.nonzero(p).flatten(), torch.nonzero(q).flatten()])
        nv = int(valid[r].sum())
        assert nv == len(want) and bool(valid[r, :nv].all())
        assert torch.equal(order[r, :nv].cpu(), want)
        assert not order[r, nv:].any()
    assert bool(pos[2, :40].all()) and bool(neg[2, 40:100].all())
    # uniformity: row 0 positives (k = 128 of n) over 400 seeds
    ispos0 = ((lc[0] != -1) & (lc[0] != bg)).to(dev)
    n0 = int(ispos0.sum())
    hits = torch.zeros(P, device=dev)
    T = 400
    for t in range(T):
        p, _ = ops().subsample(lab[:1], S, num_pos, bg, torch.tensor([t * 7919 + 1], device=dev))
        hits += p[0].float()
    f = (hits[ispos0] / T).cpu().numpy()
    pk = num_pos / n0
    sd = math.sqrt(pk * (1 - pk) / T)
    assert abs(f.mean() - pk) < 1e-6 + 1e-3  # exact k per draw
    assert (np.abs(f - pk) < 6 * sd).mean() > 0.999, (pk, f.min(), f.max())


@pytest.mark.gpu
def test_fused_subsample_pairwise_co_inclusion(dev):
    """Second-order uniformity of d2mi_subsample: with k of n kept, every pair
    of candidates must be kept together with probability k(k-1) / (n(n-1)),
    as for a uniform shuffle (tf.random_shuffle(...)[:k]).  4,000 independent
    draws (rows: each row's Feistel round keys differ), n = 40, k = 10: all
    780 pair frequencies within 5 sd, and neighbouring ranks (where a weak
    permutation would correlate) no further off on average than the rest."""
    T, n, k, bg = 4000, 40, 10, 80
    lab = torch.full((T, n), 3, dtype=torch.int64, device=dev)
    seed = torch.tensor([987654321987], dtype=torch.int64, device=dev)
    pos, neg = ops().subsample(lab, k, k, bg, seed)
    assert not neg.any()
    p = pos.double()
    assert bool((p.sum(1) == k).all())
    first = (p.sum(0) / T).cpu().numpy()
    pk = k / n
    assert np.all(np.abs(first - pk) < 5 * math.sqrt(pk * (1 - pk) / T)), first
    co = ((p.t() @ p) / T).cpu().numpy()
    p2 = k * (k - 1) / (n * (n - 1))
    sd = math.sqrt(p2 * (1 - p2) / T)
    off = co[~np.eye(n, dtype=bool)]
    assert np.all(np.abs(off - p2) < 5 * sd), (off.min(), off.max(), p2)
    near = np.array([co[i, i + 1] for i in range(n - 1)])
    assert abs(near.mean() - p2) < 5 * sd / math.sqrt(n - 1) + 1e-3, (near.mean(), p2)


def _mask_rcnn_cfg():
    from detectron2_tensorflow_amd.config import get_cfg
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(os.path.dirname(__file__), "..", "configs",
                                     "COCO-InstanceSegmentation", "mask_rcnn_R_50_FPN_1x.yaml"))
    return cfg


@pytest.mark.parametrize("case", ["mixed", "empty_gt_image", "few_proposals"])
def test_roi_sample_take_matches_torch_glue(dev, case):
    """d2mi_roi_gt_classes + d2mi_roi_sample_take (label_and_sample_proposals'
    glue and the mask branch's fg-first inputs, roi_heads.py:100-232 / :35-62)
    vs the torch form of the same steps on the same sampler draw: every
    sampled field, the six fg-first mask inputs, the foreground flags and the
    count equal (pure data movement); with crowd / difficult GT, invalid
    proposal slots, an image with no valid GT, and fewer proposals than slots."""
    from detectron2_tensorflow_amd.layers import ShapeSpec
    from detectron2_tensorflow_amd.modeling.roi_heads.roi_heads import StandardROIHeads
    from detectron2_tensorflow_amd.structures import BoxList
    cfg = _mask_rcnn_cfg()
    heads = StandardROIHeads(cfg, {f"p{i}": ShapeSpec(channels=256, stride=2 ** i)
                                   for i in range(2, 6)}).to(dev)
    rng = np.random.default_rng({"mixed": 1, "empty_gt_image": 2, "few_proposals": 3}[case])
    N, G = 2, 7
    P = 300 if case == "few_proposals" else 1000
    gt = np.stack([rand_boxes(rng, G, 800, 1333) for _ in range(N)])
    props = np.stack([rand_boxes(rng, P, 800, 1333) for _ in range(N)])
    near = rng.integers(0, G, (N, P // 3))
    props[:, :P // 3] = (np.take_along_axis(gt, near[..., None], 1)
                         + rng.normal(0, 6, (N, P // 3, 4))).astype(F32)
    pvalid = np.ones((N, P), bool)
    pvalid[1, P - 120:] = False
    gvalid = np.ones((N, G), bool)
    gvalid[0, 5:] = False
    if case == "empty_gt_image":
        gvalid[1] = False
    crowd = np.zeros((N, G), bool)
    crowd[0, 2] = True
    diff = np.zeros((N, G), bool)
    diff[1, 3] = True
    pl = BoxList(torch.from_numpy(props).to(dev))
    pl.add_field("is_valid", torch.from_numpy(pvalid).to(dev))
    targets = {"gt_boxes": torch.from_numpy(gt).to(dev),
               # (int32 GT classes in one case: the kernel reads either width)
               "gt_classes": torch.from_numpy(rng.integers(0, 80, (N, G)).astype(
                   np.int32 if case == "few_proposals" else np.int64)).to(dev),
               "is_valid": torch.from_numpy(gvalid).to(dev),
               "gt_is_crowd": torch.from_numpy(crowd).to(dev),
               "gt_difficult": torch.from_numpy(diff).to(dev),
               "gt_masks": torch.rand(N, G, 56, 56, device=dev)}
    from detectron2_tensorflow_amd.layers import ops as lops
    try:
        lops.FUSED_SAMPLE_TAKE = False
        torch.manual_seed(11)
        ref = heads.label_and_sample_proposals(pl, targets)
        lops.FUSED_SAMPLE_TAKE = True
        torch.manual_seed(11)
        got = heads.label_and_sample_proposals(pl, targets)
    finally:
        lops.FUSED_SAMPLE_TAKE = True
    fused = got.pop("_mask_prep")
    assert sorted(got) == sorted(ref)
    for k in ref:
        assert got[k].dtype == ref[k].dtype and torch.equal(got[k], ref[k]), k
    ts, _, fg = heads._mask_prep(ref, targets)
    for a, b in zip(fused[0], ts):
        assert a.dtype == b.dtype and torch.equal(a, b)
    assert torch.equal(fused[1], fg)
    assert int(fused[2].item()) == int(fg.sum().item())
    if case == "empty_gt_image":
        assert not bool(fg[fg.numel() // 2:].any())
