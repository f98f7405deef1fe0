from .build import BACKBONE_REGISTRY, Backbone, build_backbone
from .resnet import ResNet, Stem, Stage, BottleneckBlock

__all__ = ["BACKBONE_REGISTRY", "Backbone", "build_backbone", "ResNet", "Stem", "Stage",
           "BottleneckBlock"]
