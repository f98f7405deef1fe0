"""ROIPooler (lib/modeling/poolers.py:52-180).

The reference gathers boxes per level, runs one ROIAlign per level (each with
a full-map SYMMETRIC pad), concatenates and inverts the permutation.  Here a
single HIP launch assigns each box its level in-kernel (the same
assign_boxes_to_levels arithmetic, :11-49) and writes every pooled ROI
directly at its input row.
"""
import math
import sys

import torch

from ..layers import Layer
from ..layers import ops


def assign_boxes_to_levels(boxes, min_level, max_level, canonical_box_size, canonical_level):
    """poolers.py:11-49 on a [R, 4] tensor (reference for tests / CPU use)."""
    eps = sys.float_info.epsilon
    area = (boxes[:, 2] - boxes[:, 0]) * (boxes[:, 3] - boxes[:, 1])
    lv = torch.floor(canonical_level + torch.log(torch.sqrt(area) / canonical_box_size + eps)
                     / math.log(2))
    lv = torch.nan_to_num(lv, nan=min_level, posinf=min_level, neginf=min_level).to(torch.int64)
    return torch.clamp(lv, min_level, max_level) - min_level


class ROIPooler(Layer):
    def __init__(self, output_size, scales, sampling_ratio, pooler_type, canonical_box_size=224,
                 canonical_level=4, **kwargs):
        super().__init__(**kwargs)
        if isinstance(output_size, int):
            output_size = (output_size, output_size)
        assert len(output_size) == 2
        self.output_size = tuple(output_size)
        if pooler_type == "ROIAlign":
            self.aligned = False
        elif pooler_type == "ROIAlignV2":
            self.aligned = True
        else:
            raise ValueError(f"Unknown pooler type: {pooler_type}")
        self.scales = [float(s) for s in scales]
        self.sampling_ratio = int(sampling_ratio)
        min_level = -math.log2(scales[0])
        max_level = -math.log2(scales[-1])
        assert math.isclose(min_level, int(min_level)) and math.isclose(max_level, int(max_level))
        self.min_level, self.max_level = int(min_level), int(max_level)
        assert 0 < self.min_level <= self.max_level
        assert self.min_level <= canonical_level <= self.max_level
        self.canonical_level = canonical_level
        assert canonical_box_size > 0
        self.canonical_box_size = canonical_box_size

    def pool(self, x, boxes, box_img, return_levels=False, grad_share=None):
        """x: list of NHWC maps; boxes [R, 4] image px; box_img [R] image index.
        grad_share: a dict shared with another pooling of the same maps whose
        backward also runs (ops._RoIAlignFn): one gradient map set, no add."""
        assert len(x) == len(self.scales), (
            f"unequal value, num_level_assignments={len(self.scales)}, but x is list of {len(x)} Tensors")
        return ops.roi_align(x, boxes, box_img, self.output_size, self.scales, self.sampling_ratio,
                             aligned=self.aligned, min_level=self.min_level,
                             max_level=self.max_level,
                             canonical_box_size=self.canonical_box_size,
                             canonical_level=self.canonical_level, return_levels=return_levels,
                             grad_share=grad_share)

    def call(self, x, instances):
        """instances: SparseBoxList (boxes in .data, image index in .indices[:, 0])."""
        return self.pool(x, instances.data.boxes, instances.indices[:, 0])
