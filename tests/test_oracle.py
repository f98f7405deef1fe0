"""CPU tests: the oracle against the reference's golden vectors and
hand-computed known answers (no GPU)."""
import math
import os

import numpy as np
import pytest

import oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "nms_golden.npz")
F32 = np.float32


def test_nms_matches_reference_numpy_nms():
    """oracle NMS == lib/structures/np_box_list_ops.py:146-217 on every golden case."""
    d = np.load(GOLDEN)
    for i in range(int(d["num_cases"])):
        thr, max_out = d[f"c{i}_params"]
        got = oracle.nms(d[f"c{i}_boxes"], d[f"c{i}_scores"], int(max_out), float(thr))
        np.testing.assert_array_equal(got, d[f"c{i}_keep"], err_msg=f"case {i}")


def test_nms_kat_threshold_is_strict():
    # IoU(box0, box1) = 0.69, IoU(box0, box2) = 0.71: thr 0.7 keeps 0,1 and drops 2
    b0 = [0, 0, 10, 10]
    # box1: shift in x so that IoU = 0.69 -> inter = 100*(1-d/10), IoU = (10-d)/(10+d)
    d1 = 10 * (1 - 0.69) / (1 + 0.69)
    d2 = 10 * (1 - 0.71) / (1 + 0.71)
    boxes = np.array([b0, [0, d1, 10, 10 + d1], [0, d2, 10, 10 + d2]], F32)
    scores = np.array([0.9, 0.8, 0.7], F32)
    assert list(oracle.nms(boxes, scores, 10, 0.7)) == [0, 1]
    # equal IoU to the threshold is NOT suppressed (IOU > thr)
    boxes = np.array([[0, 0, 10, 10], [0, 0, 10, 5]], F32)  # IoU 0.5
    assert list(oracle.nms(boxes, np.array([1.0, 0.5], F32), 10, 0.5)) == [0, 1]


def test_nms_tie_rule_and_degenerate_boxes():
    boxes = np.array([[0, 0, 1, 1], [0, 0, 1, 1], [5, 5, 6, 6]], F32)
    # equal scores: lowest index first
    assert list(oracle.nms(boxes, np.array([0.5, 0.5, 0.1], F32), 10, 0.5)) == [0, 2]
    # zero-area boxes never suppress (IoU := 0)
    z = np.array([[1, 1, 1, 1], [1, 1, 1, 1]], F32)
    assert list(oracle.nms(z, np.array([0.9, 0.8], F32), 10, 0.0)) == [0, 1]
    # corners are min/max normalised
    flipped = np.array([[0, 0, 10, 10], [10, 10, 0, 0]], F32)
    assert list(oracle.nms(flipped, np.array([0.9, 0.8], F32), 10, 0.5)) == [0]
    # NaN / -inf scores are never selected, max_output_size caps
    s = np.array([np.nan, -np.inf, 0.3], F32)
    assert list(oracle.nms(np.array([[0, 0, 1, 1], [2, 2, 3, 3], [4, 4, 5, 5]], F32), s, 10, 0.5)) == [2]
    assert len(oracle.nms(boxes, np.array([0.5, 0.4, 0.3], F32), 1, 0.5)) == 1
    with pytest.raises(ValueError):
        oracle.nms(boxes, np.ones(3, F32), 10, 1.5)


def test_crop_and_resize_kat():
    """tf.image.crop_and_resize sample positions: in_y = y1*(H-1) + y*(y2-y1)*(H-1)/(ch-1)."""
    H, W = 5, 7
    img = (np.arange(H)[:, None] * 100 + np.arange(W)[None, :]).astype(F32)[None, :, :, None]
    box = np.array([[0.25, 0.5, 0.75, 1.0]], F32)
    out = oracle.crop_and_resize_tf(img, box, [0], (3, 4))[0, :, :, 0]
    ys = 0.25 * 4 + np.arange(3) * (0.5 * 4 / 2)
    xs = 0.5 * 6 + np.arange(4) * (0.5 * 6 / 3)
    np.testing.assert_allclose(out, ys[:, None] * 100 + xs[None, :], rtol=0, atol=1e-4)
    # outside [0, H-1] -> extrapolation value 0; crop 1 -> centre sample
    out = oracle.crop_and_resize_tf(img, np.array([[-1.0, 0, -0.5, 1]], F32), [0], (2, 2))
    assert np.all(out == 0)
    c = oracle.crop_and_resize_tf(img, np.array([[0, 0, 1, 1]], F32), [0], (1, 1))[0, 0, 0, 0]
    assert abs(c - (2 * 100 + 3)) < 1e-5
    with pytest.raises(ValueError):
        oracle.crop_and_resize_tf(img, box, [1], (2, 2))


def test_roi_align_aligned_bin_centres():
    """ROIAlignV2 with SR=0 samples bin centres: ymin*s + (i+0.5)*h*s/oh - 0.5
    (functional.py:138-152 on the SYMMETRIC-padded map)."""
    H, W = 16, 20
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    img = (yy * 1000 + xx).astype(F32)[None, :, :, None]
    box = np.array([[2.0, 3.0, 10.0, 15.0]], F32) * 4  # image px, stride 4
    out = oracle.roi_align(img, box, [0], (4, 6), 0.25, 0, aligned=True)[0, :, :, 0]
    cy = 2 + (np.arange(4) + 0.5) * 8 / 4 - 0.5
    cx = 3 + (np.arange(6) + 0.5) * 12 / 6 - 0.5
    np.testing.assert_allclose(out, cy[:, None] * 1000 + cx[None, :], rtol=0, atol=2e-3)
    # edge replicate through the SYMMETRIC pad: a box hanging off the top-left
    out = oracle.roi_align(img, np.array([[-2.0, -2.0, 2.0, 2.0]], F32), [0], (2, 2), 1.0, 0)[0, :, :, 0]
    assert out[0, 0] == img[0, 0, 0, 0]


def test_roi_align_sampling_ratio_is_mean_of_samples():
    rng = np.random.default_rng(0)
    img = rng.normal(size=(1, 12, 12, 3)).astype(F32)
    box = np.array([[8.0, 4.0, 40.0, 44.0]], F32)
    a = oracle.roi_align(img, box, [0], (2, 2), 0.25, 2)
    b = oracle.roi_align(img, box, [0], (4, 4), 0.25, 0)
    np.testing.assert_allclose(a, b.reshape(1, 2, 2, 2, 2, 3).mean(axis=(2, 4)), atol=1e-6)


def test_cell_anchor_kat():
    """size 32, ratio 0.5: w = sqrt(1024/0.5) = 45.25, h = 22.63 (anchor_generator.py:132-143)."""
    cell = oracle.generate_cell_anchors([32], [0.5, 1.0, 2.0])
    w = math.sqrt(1024 / 0.5)
    np.testing.assert_allclose(cell[0], [-0.25 * w, -w / 2, 0.25 * w, w / 2], rtol=1e-6)
    grid = oracle.grid_anchors(3, 4, 4, cell)
    assert grid.shape == (3 * 4 * 3, 4)
    # anchor k at (i, j) = cell + [4i, 4j, 4i, 4j], order [H, W, A]
    i, j, a = 2, 3, 1
    np.testing.assert_array_equal(grid[(i * 4 + j) * 3 + a], cell[a] + np.array([8, 12, 8, 12], F32))


def test_apply_deltas_identity_and_clamp():
    boxes = np.array([[10, 20, 30, 60]], F32)
    out = oracle.apply_deltas(np.zeros((1, 8), F32), boxes, (10, 10, 5, 5))
    np.testing.assert_array_equal(out.reshape(2, 4), np.repeat(boxes, 2, 0))
    big = oracle.apply_deltas(np.array([[0, 0, 100, 100]], F32), boxes, (1, 1, 1, 1))
    h = 20 * 1000 / 16
    np.testing.assert_allclose(big[0, 2] - big[0, 0], h, rtol=1e-5)


def test_assign_levels_kat():
    # sqrt(area) = 224 -> canonical level 4 -> index 2 of [2..5]
    b = np.array([[0, 0, 224, 224], [0, 0, 112, 112], [0, 0, 10, 10], [0, 0, 2000, 2000],
                  [0, 0, 0, 0]], F32)
    lv = oracle.assign_boxes_to_levels(b, 2, 5, 224, 4)
    assert list(lv) == [2, 1, 0, 3, 0]


def test_top_k_order():
    v = np.array([1.0, 3.0, 3.0, -1.0, 2.0], F32)
    vals, idx = oracle.top_k(v, 3)
    assert list(idx) == [1, 2, 4] and list(vals) == [3.0, 3.0, 2.0]


def test_matrix_nms_kat():
    m = np.zeros((3, 4, 4), F32)
    m[0, :2, :2] = 1
    m[1, :2, :3] = 1   # overlaps mask 0: inter 4, union 6 -> iou 2/3
    m[2, 2:, 2:] = 1
    out = oracle.matrix_nms(m, np.array([0, 0, 0]), np.array([0.9, 0.8, 0.7], F32))
    iou = 4 / 6
    np.testing.assert_allclose(out, [0.9, 0.8 * math.exp(-2 * iou ** 2), 0.7], rtol=1e-6)


def test_paste_masks_kat_in_range_region():
    """reframe_box_masks_to_image_masks (mask_ops.py:35-56): with a constant box
    mask above the threshold, a canvas pixel is set iff crop_and_resize samples
    inside the mask, i.e. 0 <= (mh-1) * (y/(H-1) - y1/H) / ((y2-y1)/H) <= mh-1
    (note the canvas is normalised by H but sampled on H-1 steps), same for x."""
    H, W, mh = 60, 80, 28
    box = np.array([[12.0, 20.0, 40.0, 61.0]], np.float32)
    out = oracle.paste_masks(np.full((1, mh, mh), 0.9, np.float32), box, (H, W))[0]

    def inside(n, c1, c2):
        t = (mh - 1) * (np.arange(n) / (n - 1) - c1 / n) / ((c2 - c1) / n)
        return (t >= 0) & (t <= mh - 1), np.minimum(np.abs(t), np.abs(t - (mh - 1)))

    iy, dy = inside(H, 12.0, 40.0)
    ix, dx = inside(W, 20.0, 61.0)
    want = (iy[:, None] & ix[None, :]).astype(np.uint8)
    safe = (dy[:, None] > 1e-3) & (dx[None, :] > 1e-3)
    np.testing.assert_array_equal(out[safe], want[safe])
    # invalid rows are zero; threshold is strict
    z = oracle.paste_masks(np.full((2, mh, mh), 0.5, np.float32), np.repeat(box, 2, 0), (H, W),
                           valid=np.array([True, False]))
    assert z.sum() == 0


# ------------------------------------------------ reference-held box-op goldens
BOX_GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "box_ops_golden.npz")


def test_pairwise_iou_matches_reference_numpy_iou():
    """oracle/training.py pairwise_iou (the TF box_list_ops formula, float32)
    vs the reference's np_box_ops.iou (np_box_ops.py:48-63, float64
    intersection): equal to float32 rounding; the matcher decisions on the
    two matrices are identical (tie- and threshold-safe inputs)."""
    import training
    g = np.load(BOX_GOLDEN)
    ours = training.pairwise_iou(g["iou_gt"], g["iou_boxes"])
    np.testing.assert_allclose(ours, g["iou"], rtol=2e-6, atol=1e-7)
    for thr, labels in (((0.3, 0.7), (0, -1, 1)), ((0.5,), (0, 1))):
        m1, l1 = training.matcher(ours, thr, labels, True)
        m2, l2 = training.matcher(g["iou"].astype(np.float32), thr, labels, True)
        np.testing.assert_array_equal(m1, m2)
        np.testing.assert_array_equal(l1, l2)
    assert len(set(l1.tolist())) == 2 and (l1 == 1).sum() > 100


def test_clip_to_window_matches_reference_numpy_clip():
    """clip_to_window (box_list_ops.py:112-147) vs np_box_list_ops.clip_to_window
    (np_box_list_ops.py:319-350): identical clipped corners; the reference's
    numpy version then drops zero-area boxes (the TF op with
    filter_nonoverlapping=True does the same)."""
    g = np.load(BOX_GOLDEN)
    out = oracle.clip_to_window(g["clip_boxes"], g["clip_window"])
    area = (out[:, 2] - out[:, 0]) * (out[:, 3] - out[:, 1])
    keep = np.nonzero(area > 0)[0]
    np.testing.assert_array_equal(keep, g["clip_keep"])
    np.testing.assert_array_equal(out[keep], g["clip_out"])


def test_apply_deltas_matches_reference_numpy_decode():
    """Box2BoxTransform.apply_deltas with weights (1, 1, 1, 1) vs the reference's
    np_box_ops.apply_box_deltas (np_box_ops.py:85-113): the same decode up to
    rounding (numpy forms ymax = ymin + h, the transform cy + h / 2)."""
    g = np.load(BOX_GOLDEN)
    got = oracle.apply_deltas(g["dec_deltas"], g["dec_boxes"], (1, 1, 1, 1))
    want = g["dec_out"]
    tol = np.maximum(np.float32(1e-4), 4 * np.spacing(np.abs(want).max(axis=1, keepdims=True)))
    assert (np.abs(got - want) <= tol).all()


MC_GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "multiclass_nms_golden.npz")


def test_fast_rcnn_inference_matches_reference_multiclass_nms():
    """oracle.fast_rcnn_inference (class-offset NMS, fast_rcnn.py:141-145) on
    one class-agnostic box per ROI == the reference's numpy
    multi_class_non_max_suppression (np_box_list_ops.py:220-290) on the same
    boxes and softmax scores (tests/golden/multiclass_nms_golden.npz: inputs
    where the offset trick cannot change an IoU decision)."""
    g = np.load(MC_GOLDEN)
    boxes, logits = g["mc_boxes"], g["mc_logits"]
    thr, score_thresh = g["mc_params"]
    R, K = logits.shape[0], logits.shape[1] - 1
    probs = oracle.softmax(logits)
    np.testing.assert_array_equal(probs[:, :K][probs[:, :K] > score_thresh].size,
                                  (probs[:, :K] > score_thresh).sum())
    res = oracle.fast_rcnn_inference(np.tile(boxes, (1, K)), probs, np.zeros(R, np.int64),
                                     np.arange(R), R, [(1000, 1000)], score_thresh, thr, 100)
    ob, osc, oc, ov, oroi = res[0]
    n = int(ov.sum())
    assert n == len(g["mc_sel_rows"])
    np.testing.assert_array_equal(oroi[:n], g["mc_sel_rows"])
    np.testing.assert_array_equal(oc[:n], g["mc_sel_classes"])
    np.testing.assert_array_equal(osc[:n], g["mc_sel_scores"])
    np.testing.assert_array_equal(ob[:n], g["mc_sel_boxes"])


# ------------------------------------------------ reference-held VOC metrics goldens
VOC_GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "voc_metrics_golden.npz")


def test_voc_metrics_match_reference_metrics():
    """evaluation/voc_metrics == lib/evaluation/metrics.py:7-95 (the
    reference's own compute_precision_recall / compute_average_precision,
    tests/golden/voc_metrics_golden.npz) bit for bit, bool and weighted
    labels, a class without detections; num_gt == 0 -> (None, None) -> NaN."""
    from detectron2_tensorflow_amd.evaluation import voc_metrics
    d = np.load(VOC_GOLDEN)
    for i in range(int(d["num_cases"])):
        p, r = voc_metrics.precision_recall(d[f"v{i}_scores"], d[f"v{i}_labels"],
                                            int(d[f"v{i}_num_gt"]))
        np.testing.assert_array_equal(p, d[f"v{i}_precision"])
        np.testing.assert_array_equal(r, d[f"v{i}_recall"])
        assert voc_metrics.average_precision(p, r) == float(d[f"v{i}_ap"])
    p, r = voc_metrics.precision_recall(np.array([0.5]), np.array([False]), 0)
    assert p is None and r is None and math.isnan(voc_metrics.average_precision(p, r))
