"""batch_nms / matrix_nms (lib/layers/nms.py:6-83) on the gfx950 kernels."""
import torch

from . import ops


def batch_nms(boxes, scores, max_output_size, axis=0, iou_threshold=0.5, scope=None):
    """Per-row TF NonMaxSuppressionV3 in one segmented launch.

    boxes [B, N, 4] (or [N, B, 4] when axis == 0, as in the reference, which
    transposes), scores [B, N] ([N, B]).  Returns int32 [B, max_output_size]
    selected indices per row.  Deviation, documented: rows that keep fewer
    than max_output_size boxes are padded with -1 (the reference's map_fn
    would fail on ragged rows, nms.py:25)."""
    assert boxes.dim() == 3 and scores.dim() == 2
    assert axis in (0, 1)
    if axis == 0:
        boxes = boxes.transpose(0, 1)
        scores = scores.transpose(0, 1)
    B, N = scores.shape
    off = torch.arange(0, (B + 1) * N, N, dtype=torch.int32, device=boxes.device)
    keep, _ = ops.nms_segments(boxes.reshape(-1, 4), scores.reshape(-1), off, max_output_size,
                               iou_threshold, seg_capacity=N)
    return keep


def matrix_nms(masks, classes, scores, sum_masks=None, kernel="gaussian", sigma=2.0, scope=None):
    """SOLOv2 Matrix-NMS: masks [N, H, W], classes [N], scores [N] -> decayed scores [N]."""
    assert masks.dim() == 3 and classes.dim() == 1 and scores.dim() == 1
    return ops.matrix_nms_scores(masks, classes, scores, sum_masks, kernel, sigma)
