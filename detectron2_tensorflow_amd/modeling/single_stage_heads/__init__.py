from .build import SINGLE_STAGE_HEADS_REGISTRY, build_single_stage_head
from .retinanet import RetinaNetBoxTower, RetinaNetHead
from .solo_v2 import MaskFeatureBranch, MaskKernelBranch, SOLOv2Head

__all__ = ["SINGLE_STAGE_HEADS_REGISTRY", "build_single_stage_head", "RetinaNetHead",
           "RetinaNetBoxTower", "SOLOv2Head", "MaskKernelBranch", "MaskFeatureBranch"]
