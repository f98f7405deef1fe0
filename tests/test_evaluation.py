"""COCO bbox AP restatement (pycocotools COCOeval, bbox): known answers."""
import numpy as np
import pytest

from detectron2_tensorflow_amd.evaluation import COCOBoxEvaluator


def test_perfect_detections_give_ap_100():
    ev = COCOBoxEvaluator()
    gt = np.array([[10, 10, 60, 80], [100, 120, 200, 300]], float)
    ev.add(gt, [1, 2], gt, [0.9, 0.8], [1, 2])
    r = ev.summarize()
    assert r["AP"] == pytest.approx(100.0) and r["AP50"] == pytest.approx(100.0)
    assert r["APs"] == -1.0 and r["APl"] == pytest.approx(100.0)


def test_false_positive_ranked_first_halves_precision():
    """One GT, a higher-scored miss then a hit: precision 0 then 1/2, made
    monotone -> 1/2 at every recall point -> AP 50 (at every IoU threshold)."""
    ev = COCOBoxEvaluator()
    gt = np.array([[0, 0, 100, 100]], float)
    ev.add(gt, [3], [[200, 200, 300, 300], [0, 0, 100, 100]], [0.9, 0.5], [3, 3])
    assert ev.summarize()["AP"] == pytest.approx(50.0, abs=1e-6)


def test_iou_threshold_sweep():
    """A detection at IoU 0.709 (x shifted) is a hit for thresholds 0.50..0.70 only:
    5 of 10 -> AP 50, AP50 100, AP75 0."""
    ev = COCOBoxEvaluator()
    # GT 0..100 x 0..100; det 0..100 x s..100+s: IoU (100-s)/(100+s)
    s = 17.0  # IoU = 83 / 117 = 0.709
    ev.add([[0, 0, 100, 100]], [0], [[0, s, 100, 100 + s]], [0.7], [0])
    r = ev.summarize()
    assert r["AP"] == pytest.approx(50.0, abs=1e-6)
    assert r["AP50"] == pytest.approx(100.0) and r["AP75"] == pytest.approx(0.0)


def test_crowd_gt_is_ignored_and_absorbs_matches():
    """A detection on a crowd region is neither TP nor FP; the real object
    still needs its own detection."""
    ev = COCOBoxEvaluator()
    gt = [[0, 0, 50, 50], [100, 100, 300, 300]]
    ev.add(gt, [1, 1], [[120, 120, 180, 180], [0, 0, 50, 50]], [0.95, 0.6], [1, 1],
           gt_crowd=[False, True])
    assert ev.summarize()["AP"] == pytest.approx(100.0)


def test_unmatched_class_and_missing_detections():
    ev = COCOBoxEvaluator()
    ev.add([[0, 0, 40, 40], [0, 50, 40, 90]], [1, 2], [[0, 0, 40, 40]], [0.9], [1])
    # class 1 perfect, class 2 never detected -> mean of 100 and 0
    assert ev.summarize()["AP"] == pytest.approx(50.0)
