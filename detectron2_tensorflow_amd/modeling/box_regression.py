"""Box2BoxTransform (lib/modeling/box_regression.py:13-123), deltas (dy, dx, dh, dw)."""
import math

import torch

from ..layers import ops

_DEFAULT_SCALE_CLAMP = math.log(1000.0 / 16)


class Box2BoxTransform:
    def __init__(self, weights, scale_clamp=_DEFAULT_SCALE_CLAMP):
        self.weights = tuple(float(w) for w in weights)
        self.scale_clamp = scale_clamp

    def get_deltas(self, src_boxes, target_boxes):
        """box_regression.py:38-74 (training targets)."""
        sh = src_boxes[:, 2] - src_boxes[:, 0]
        sw = src_boxes[:, 3] - src_boxes[:, 1]
        scy = src_boxes[:, 0] + 0.5 * sh
        scx = src_boxes[:, 1] + 0.5 * sw
        th = target_boxes[:, 2] - target_boxes[:, 0]
        tw = target_boxes[:, 3] - target_boxes[:, 1]
        tcy = target_boxes[:, 0] + 0.5 * th
        tcx = target_boxes[:, 1] + 0.5 * tw
        wy, wx, wh, ww = self.weights
        dy = wy * (tcy - scy) / sh
        dx = wx * (tcx - scx) / sw
        dh = wh * torch.log(th / sh)
        dw = ww * torch.log(tw / sw)
        return torch.stack([dy, dx, dh, dw], dim=1)

    def apply_deltas(self, deltas, boxes):
        """deltas [N, K*4], boxes [N, 4] -> [N, K*4] on the HIP decode kernel."""
        return ops.apply_deltas(deltas, boxes, self.weights, self.scale_clamp)
