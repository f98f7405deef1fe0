"""BACKBONE_REGISTRY / build_backbone (lib/modeling/backbone/build.py)."""
from ...layers import Layer, ShapeSpec
from ...layers.convolutional import FoldGroup
from ...utils.registry import Registry

BACKBONE_REGISTRY = Registry("BACKBONE")


class Backbone(Layer):
    """Base: ``call(images NHWC) -> dict[name -> NHWC map]`` plus output_shape()."""

    @property
    def size_divisibility(self):
        return 0

    def output_shape(self):
        return {name: ShapeSpec(channels=self._out_feature_channels[name],
                                stride=self._out_feature_strides[name])
                for name in self._out_features}


def build_backbone(cfg, input_shape=None, **kwargs):
    if input_shape is None:
        input_shape = ShapeSpec(channels=len(cfg.MODEL.PIXEL_MEAN))
    backbone = BACKBONE_REGISTRY.get(cfg.MODEL.BACKBONE.NAME)(cfg, input_shape, **kwargs)
    if FoldGroup.ENABLED:
        FoldGroup.attach(backbone)  # its BN-convs fold in one batch per training step
    return backbone
