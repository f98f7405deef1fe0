from .build import SINGLE_STAGE_HEADS_REGISTRY, build_single_stage_head
from .retinanet import RetinaNetBoxTower, RetinaNetHead

__all__ = ["SINGLE_STAGE_HEADS_REGISTRY", "build_single_stage_head", "RetinaNetHead",
           "RetinaNetBoxTower"]
