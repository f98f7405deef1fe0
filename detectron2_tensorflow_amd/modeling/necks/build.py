"""NECK_REGISTRY / build_neck / DummyNeck (lib/modeling/necks/build.py:7-85)."""
from ...layers import Layer
from ...utils.registry import Registry

NECK_REGISTRY = Registry("NECK")


class DummyNeck(Layer):
    """Identity neck used when MODEL.NECK.NAME is empty."""

    def __init__(self, input_shape, **kwargs):
        super().__init__(**kwargs)
        self._shape = input_shape

    @property
    def size_divisibility(self):
        return 0

    def output_shape(self):
        return self._shape

    def call(self, x):
        return x


def build_neck(cfg, input_shape, **kwargs):
    name = cfg.MODEL.NECK.NAME
    if not name:
        return DummyNeck(input_shape, **kwargs)
    return NECK_REGISTRY.get(name)(cfg, input_shape, **kwargs)
