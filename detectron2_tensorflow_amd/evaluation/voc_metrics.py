"""Pascal-VOC precision / recall and average precision, restating the
reference's lib/evaluation/metrics.py:7-95 (compute_precision_recall,
compute_average_precision), the arithmetic its pascal_voc_evaluator.py:573-589
runs per class and for the mean AP.  Pinned bit for bit against the
reference's own numpy functions (tests/golden/make_golden.py ->
voc_metrics_golden.npz, tests/test_oracle.py).
"""
import numpy as np


def precision_recall(scores, labels, num_gt):
    """metrics.py:7-47.  scores [N] float, labels [N] bool / float
    (true-positive weights), num_gt: positives.  Detections in descending
    score order (the reference's argsort()[::-1]: ties in reverse index
    order); precision = cum TP / (cum TP + cum FP), recall = cum TP / num_gt.
    (None, None) when num_gt == 0."""
    scores = np.asarray(scores)
    labels = np.asarray(labels)
    if labels.ndim != 1 or scores.ndim != 1:
        raise ValueError("scores and labels must be single dimension numpy arrays")
    if labels.dtype != np.float64 and labels.dtype != np.bool_:
        raise ValueError("labels type must be either bool or float")
    if num_gt < np.sum(labels):
        raise ValueError("Number of true positives must be smaller than num_gt.")
    if len(scores) != len(labels):
        raise ValueError("scores and labels must be of the same size.")
    if num_gt == 0:
        return None, None
    order = np.argsort(scores)[::-1]
    tp = labels[order]
    fp = (tp <= 0).astype(float)
    ctp = np.cumsum(tp)
    cfp = np.cumsum(fp)
    return ctp.astype(float) / (ctp + cfp), ctp.astype(float) / num_gt


def average_precision(precision, recall):
    """metrics.py:50-95 (VOCdevkit): precision made non-increasing from the
    right over recall padded with 0 / 1, summed over the recall steps.  NaN
    when precision is None."""
    if precision is None:
        if recall is not None:
            raise ValueError("If precision is None, recall must also be None")
        return np.nan
    precision = np.asarray(precision)
    recall = np.asarray(recall)
    if precision.dtype != np.float64 or recall.dtype != np.float64:
        raise ValueError("input must be float numpy array.")
    if len(precision) != len(recall):
        raise ValueError("precision and recall must be of the same size.")
    if not precision.size:
        return 0.0
    if precision.min() < 0 or precision.max() > 1:
        raise ValueError("Precision must be in the range of [0, 1].")
    if recall.min() < 0 or recall.max() > 1:
        raise ValueError("recall must be in the range of [0, 1].")
    if np.any(recall[1:] < recall[:-1]):
        raise ValueError("recall must be a non-decreasing array")
    r = np.concatenate([[0], recall, [1]])
    p = np.concatenate([[0], precision, [0]])
    p = np.maximum.accumulate(p[::-1])[::-1]
    idx = np.nonzero(r[1:] != r[:-1])[0] + 1
    return np.sum((r[idx] - r[idx - 1]) * p[idx])
