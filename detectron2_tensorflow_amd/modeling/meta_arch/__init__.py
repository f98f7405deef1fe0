from .build import META_ARCH_REGISTRY, build_model
from .rcnn import GeneralizedRCNN, ProposalNetwork
from .single_stage_detector import SingleStageDetector

__all__ = ["META_ARCH_REGISTRY", "build_model", "GeneralizedRCNN", "ProposalNetwork",
           "SingleStageDetector"]
