"""GPU parity at the BASELINE geometry (SURVEY.md section 8, C2 / C3 at
1333x800, padded to 800x1344) and against the reference-held numpy goldens.

* ROIAlign on p2..p5 [2, 200x336 ... 25x42, 256] with 1,000 ROIs per image
  (SURVEY D2 box distribution), 7x7 and 14x14, vs the oracle's per-level
  ROIPooler; level assignment: every box whose level differs from the
  oracle's is a log-boundary box (its 4 + log2(sqrt(area) / 224) lies within
  1e-5 of an integer: logf rounding on either side), and its output equals
  the oracle's ROIAlign on the level the GPU chose.
* find_top_rpn_proposals over all 268,569 anchors per image, pre / post
  1000 / 1000 (test) and 2000 / 1000 (train): kept scores and valid flags
  bit-exact, boxes within max(1e-4, 2 ulp).
* fast_rcnn_inference with R = 1,000 proposals per image, 81 classes.
* batch_nms (lib/layers/nms.py:6-26) through detectron2_tensorflow_amd.layers,
  axis 0 and 1, ragged survivors padded with -1.
* The fused matcher (d2mi_match_boxes) against the Matcher applied to the
  reference's own np_box_ops.iou matrix, and the decode against
  np_box_ops.apply_box_deltas (tests/golden/box_ops_golden.npz).
"""
import math
import os

import numpy as np
import pytest
import torch

import oracle
from test_gpu_ops import assert_boxes_close, rand_boxes

pytestmark = pytest.mark.gpu
F32 = np.float32
BOX_GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "box_ops_golden.npz")
H, W, TH, TW = 800, 1344, 800, 1333   # padded tensor / true image


def _ops():
    from detectron2_tensorflow_amd.layers import ops
    return ops


def _d2_boxes(rng, n):
    """centres ~ U(image), sqrt-area log-uniform [16, 800], aspect [0.5, 2]."""
    c = rng.uniform([0, 0], [TH, TW], size=(n, 2))
    s = np.exp(rng.uniform(np.log(16), np.log(800), size=n))
    ar = np.exp(rng.uniform(np.log(0.5), np.log(2.0), size=n))
    h, w = s * np.sqrt(ar), s / np.sqrt(ar)
    return np.stack([c[:, 0] - h / 2, c[:, 1] - w / 2, c[:, 0] + h / 2, c[:, 1] + w / 2],
                    1).astype(F32)


# ------------------------------------------------------------------ ROIAlign
@pytest.fixture(scope="module")
def fpn_levels():
    rng = np.random.default_rng(101)
    strides = [4, 8, 16, 32]
    feats = [rng.normal(size=(2, H // s, W // s, 256)).astype(F32) for s in strides]
    boxes = np.concatenate([_d2_boxes(rng, 1000), _d2_boxes(rng, 1000)])
    bimg = np.repeat(np.arange(2, dtype=np.int32), 1000)
    return feats, boxes, bimg, [1.0 / s for s in strides]


@pytest.mark.parametrize("oh", [7, 14])
def test_roi_align_baseline_geometry(dev, fpn_levels, oh):
    feats, boxes, bimg, scales = fpn_levels
    assert [f.shape[1:3] for f in feats] == [(200, 336), (100, 168), (50, 84), (25, 42)]
    want, lv_want = oracle.roi_pooler(feats, boxes, bimg, (oh, oh), scales, 0, True)
    got, lv = _ops().roi_align([torch.from_numpy(f).to(dev) for f in feats],
                               torch.from_numpy(boxes).to(dev), torch.from_numpy(bimg).to(dev),
                               (oh, oh), scales, 0, True, return_levels=True)
    got, lv = got.cpu().numpy(), lv.cpu().numpy()
    same = lv == lv_want
    np.testing.assert_allclose(got[same], want[same], rtol=0, atol=1e-5)
    b = boxes.astype(np.float64)
    v = 4 + np.log(np.sqrt((b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])) / 224 + 2.0 ** -52) / math.log(2)
    for i in np.nonzero(~same)[0]:
        assert abs(v[i] - round(v[i])) < 1e-5, (i, v[i], lv[i], lv_want[i])
        w1 = oracle.roi_align(feats[lv[i]], boxes[i:i + 1], bimg[i:i + 1], (oh, oh), scales[lv[i]],
                              0, True)
        np.testing.assert_allclose(got[i:i + 1], w1, rtol=0, atol=1e-5)
    assert np.bincount(lv, minlength=4).min() > 50  # every level exercised


# ------------------------------------------------------------ RPN proposals
@pytest.mark.parametrize("pre,post", [(1000, 1000), (2000, 1000)])
def test_rpn_proposals_baseline_geometry(dev, pre, post):
    rng = np.random.default_rng(202)
    N, A = 2, 3
    strides = [4, 8, 16, 32, 64]
    hw = [(int(math.ceil(H / s)), int(math.ceil(W / s))) for s in strides]
    assert sum(h * w * A for h, w in hw) == 268569
    cells = [oracle.generate_cell_anchors([sz], [0.5, 1.0, 2.0]) for sz in [32, 64, 128, 256, 512]]
    logits = [rng.normal(size=(N, h, w, A)).astype(F32) for h, w in hw]
    deltas = [rng.normal(0, 0.1, size=(N, h, w, A * 4)).astype(F32) for h, w in hw]
    image_hw = np.array([[TH, TW], [TH, TW]], np.int32)
    props = []
    for (h, w), s, c, d in zip(hw, strides, cells, deltas):
        anc = oracle.grid_anchors(h, w, s, c)
        props.append(oracle.apply_deltas(d.reshape(-1, 4), np.tile(anc, (N, 1)), (1, 1, 1, 1))
                     .reshape(N, -1, 4))
    wb, ws, wv = oracle.find_top_rpn_proposals(props, [l.reshape(N, -1) for l in logits],
                                               image_hw, 0.7, pre, post, 0.0)
    gb, gs, gv = _ops().rpn_proposals([torch.from_numpy(l).to(dev) for l in logits],
                                      [torch.from_numpy(d).to(dev) for d in deltas], strides,
                                      [torch.from_numpy(c) for c in cells],
                                      torch.from_numpy(image_hw).to(dev), pre, post, 0.7, 0.0)
    np.testing.assert_array_equal(gv.cpu().numpy(), wv)
    np.testing.assert_array_equal(gs.cpu().numpy(), ws)
    assert_boxes_close(gb.cpu().numpy(), wb)
    assert wv.sum() == N * post


# ------------------------------------------------------------- Fast R-CNN
@pytest.mark.parametrize("nms_cls_agnostic", [False, True])
def test_fast_rcnn_inference_baseline_geometry(dev, nms_cls_agnostic):
    """nms_cls_agnostic=True: ROI_HEADS.NMS_CLS_AGNOSTIC (fast_rcnn.py:138-139),
    one plain NMS over every class's filtered boxes."""
    rng = np.random.default_rng(303)
    N, P, K = 2, 1000, 80
    image_hw = np.array([[TH, TW], [TH, TW]], np.int32)
    roi_img = np.repeat(np.arange(N, dtype=np.int32), P)
    roi_slot = np.tile(np.arange(P, dtype=np.int32), N)
    props = np.concatenate([_d2_boxes(rng, P) for _ in range(N)])
    props = oracle.clip_to_window(props, [0, 0, TH, TW])
    logits = rng.normal(0, 3, size=(N * P, K + 1)).astype(F32)
    deltas = rng.normal(0, 0.5, size=(N * P, K * 4)).astype(F32)
    w = (10.0, 10.0, 5.0, 5.0)
    probs = oracle.softmax(logits)
    boxes = oracle.apply_deltas(deltas, props, w)
    want = oracle.fast_rcnn_inference(boxes, probs, roi_img, roi_slot, P, image_hw, 0.05, 0.5, 100,
                                      nms_cls_agnostic)
    gb, gs, gc, gv, groi = _ops().fast_rcnn_inference(
        torch.from_numpy(logits).to(dev), torch.from_numpy(deltas).to(dev),
        torch.from_numpy(props).to(dev), torch.from_numpy(roi_img).to(dev),
        torch.from_numpy(roi_slot).to(dev), N, P, torch.from_numpy(image_hw).to(dev), w, 0.05,
        0.5, 100, nms_cls_agnostic=nms_cls_agnostic)
    assert int((probs[:, :-1] > 0.05).sum()) > 5000  # ~3.8 (box, class) survivors per ROI
    for n in range(N):
        wb, wsc, wc, wv, wroi = want[n]
        np.testing.assert_array_equal(gv[n].cpu().numpy(), wv)
        np.testing.assert_array_equal(gc[n].cpu().numpy(), wc)
        np.testing.assert_array_equal(groi[n].cpu().numpy(), wroi)
        np.testing.assert_allclose(gs[n].cpu().numpy(), wsc, rtol=2e-6, atol=1e-7)
        assert_boxes_close(gb[n].cpu().numpy(), wb)


# ---------------------------------------------------------------- batch_nms
@pytest.mark.parametrize("axis", [0, 1])
def test_batch_nms_layer_api(dev, axis):
    """layers.batch_nms(boxes, scores, max_output_size, axis, iou_threshold):
    rows per image (axis=1: [B, N, 4]; axis=0: [N, B, 4], transposed as the
    reference does, nms.py:14-16), each row == TF NMS of that row, -1 padded."""
    from detectron2_tensorflow_amd.layers import batch_nms
    rng = np.random.default_rng(404)
    B, N, max_out = 3, 400, 50
    boxes = np.stack([rand_boxes(rng, N, 300, 400, 4, 150) for _ in range(B)])
    scores = rng.uniform(size=(B, N)).astype(F32)
    boxes[2, :, 2:] = boxes[2, :, :2] + 1000  # one row with few survivors (< max_out)
    bt, st = torch.from_numpy(boxes).to(dev), torch.from_numpy(scores).to(dev)
    if axis == 0:
        bt, st = bt.transpose(0, 1).contiguous(), st.transpose(0, 1).contiguous()
    keep = batch_nms(bt, st, max_out, axis=axis, iou_threshold=0.5).cpu().numpy()
    assert keep.shape == (B, max_out) and keep.dtype == np.int32
    for b in range(B):
        want = oracle.nms(boxes[b], scores[b], max_out, 0.5)
        np.testing.assert_array_equal(keep[b, :len(want)], want)
        assert (keep[b, len(want):] == -1).all()
    assert (keep[2] == -1).any()


# ------------------------------------------------- reference numpy goldens
def test_match_boxes_vs_reference_numpy_iou(dev):
    """d2mi_match_boxes (fused IoU + Matcher) == the Matcher on the reference's
    own np_box_ops.iou matrix: RPN thresholds (0.3, 0.7) with low-quality
    matches, ROI-head threshold 0.5."""
    import training
    g = np.load(BOX_GOLDEN)
    gt = torch.from_numpy(g["iou_gt"][None]).to(dev)
    flags = torch.ones((1, gt.shape[1]), dtype=torch.int32, device=dev)
    bx = torch.from_numpy(g["iou_boxes"]).to(dev)
    for thr, labels, lowq in (((0.3, 0.7), (0, -1, 1), True), ((0.5,), (0, 1), False)):
        m, lab = _ops().match_boxes(gt, flags, bx, [-math.inf, *thr, math.inf], labels, lowq)
        wm, wl = training.matcher(g["iou"].astype(F32), thr, labels, lowq)
        np.testing.assert_array_equal(lab[0].cpu().numpy(), wl)
        pos = wl != 0
        np.testing.assert_array_equal(m[0].cpu().numpy()[pos], wm[pos])


def test_apply_deltas_vs_reference_numpy_decode(dev):
    g = np.load(BOX_GOLDEN)
    got = _ops().apply_deltas(torch.from_numpy(g["dec_deltas"]).to(dev),
                              torch.from_numpy(g["dec_boxes"]).to(dev), (1, 1, 1, 1)).cpu().numpy()
    want = g["dec_out"]
    tol = np.maximum(F32(1e-4), 4 * np.spacing(np.abs(want).max(axis=1, keepdims=True)))
    assert (np.abs(got - want) <= tol).all()


def test_fast_rcnn_inference_vs_reference_multiclass_nms(dev):
    """The HIP fast_rcnn_inference (softmax + decode + clip + threshold +
    class-offset NMS) on one class-agnostic box per ROI (zero deltas, boxes
    inside the image) == the reference's numpy multi_class_non_max_suppression
    (np_box_list_ops.py:220-290) of the same boxes and softmax scores
    (tests/golden/multiclass_nms_golden.npz, offset-safe inputs): the same
    ROIs, classes and order; scores within the softmax's expf ulps."""
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "multiclass_nms_golden.npz"))
    boxes, logits = g["mc_boxes"], g["mc_logits"]
    thr, score_thresh = g["mc_params"]
    R = boxes.shape[0]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    gb, gs, gc, gv, groi = _ops().fast_rcnn_inference(
        t(logits), t(np.zeros((R, 4), F32)), t(boxes), t(np.zeros(R, np.int32)),
        t(np.arange(R, dtype=np.int32)), 1, R, t(np.array([[1000, 1000]], np.int32)),
        (10.0, 10.0, 5.0, 5.0), float(score_thresh), float(thr), 100, cls_agnostic=True)
    n = int(gv[0].sum())
    assert n == len(g["mc_sel_rows"])
    np.testing.assert_array_equal(groi[0, :n].cpu().numpy(), g["mc_sel_rows"])
    np.testing.assert_array_equal(gc[0, :n].cpu().numpy(), g["mc_sel_classes"])
    np.testing.assert_allclose(gs[0, :n].cpu().numpy(), g["mc_sel_scores"], rtol=2e-6, atol=1e-7)
    assert_boxes_close(gb[0, :n].cpu().numpy(), g["mc_sel_boxes"])
