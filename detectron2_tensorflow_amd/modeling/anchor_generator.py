"""DefaultAnchorGenerator (lib/modeling/anchor_generator.py:44-162).

Cell anchors are computed exactly as the reference (python float64, then
float32); ``grid_anchors`` materialises [H*W*A, 4] with the HIP kernel
d2mi_grid_anchors for API parity and for training-time matching.  The
inference hot path never materialises anchors: the fused proposal kernels
regenerate each selected anchor from its flat index.
"""
import math

import torch

from ..layers import Layer
from ..layers import ops
from ..structures import BoxList
from ..utils.registry import Registry

ANCHOR_GENERATOR_REGISTRY = Registry("ANCHOR_GENERATOR")


def generate_cell_anchors(sizes=(32, 64, 128, 256, 512), aspect_ratios=(0.5, 1, 2)):
    """anchor_generator.py:111-144: yxyx, sizes outer, ratios inner."""
    anchors = []
    for size in sizes:
        area = size ** 2.0
        for aspect_ratio in aspect_ratios:
            w = math.sqrt(area / aspect_ratio)
            h = aspect_ratio * w
            anchors.append([-h / 2.0, -w / 2.0, h / 2.0, w / 2.0])
    return torch.tensor(anchors, dtype=torch.float32)


@ANCHOR_GENERATOR_REGISTRY.register()
class DefaultAnchorGenerator(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        self.sizes = list(cfg.MODEL.ANCHOR_GENERATOR.SIZES)
        self.aspect_ratios = list(cfg.MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS)
        self.strides = [x.stride for x in input_shape]
        self.num_features = len(self.strides)
        if len(self.sizes) == 1:
            self.sizes = self.sizes * self.num_features
        if len(self.aspect_ratios) == 1:
            self.aspect_ratios = self.aspect_ratios * self.num_features
        assert self.num_features == len(self.sizes)
        assert self.num_features == len(self.aspect_ratios)
        self.cell_anchors = [generate_cell_anchors(s, a) for s, a in zip(self.sizes, self.aspect_ratios)]

    @property
    def box_dim(self):
        return 4

    @property
    def num_cell_anchors(self):
        return [c.shape[0] for c in self.cell_anchors]

    def grid_anchors(self, grid_sizes, device):
        return [ops.grid_anchors(h, w, s, c, device)
                for (h, w), s, c in zip(grid_sizes, self.strides, self.cell_anchors)]

    def call(self, features):
        grid_sizes = [(f.shape[1], f.shape[2]) for f in features]
        return [BoxList(a) for a in self.grid_anchors(grid_sizes, features[0].device)]


def build_anchor_generator(cfg, input_shape):
    return ANCHOR_GENERATOR_REGISTRY.get(cfg.MODEL.ANCHOR_GENERATOR.NAME)(cfg, input_shape)
