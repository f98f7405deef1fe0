from .build import NECK_REGISTRY, DummyNeck, build_neck
from .fpn import FPN, LastLevelMaxPool, LastLevelP6P7

__all__ = ["NECK_REGISTRY", "build_neck", "DummyNeck", "FPN", "LastLevelMaxPool", "LastLevelP6P7"]
