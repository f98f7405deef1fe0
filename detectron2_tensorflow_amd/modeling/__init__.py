"""Model surface of lib/modeling: registries, build_model and the components."""
from .anchor_generator import ANCHOR_GENERATOR_REGISTRY, DefaultAnchorGenerator, build_anchor_generator
from .backbone import BACKBONE_REGISTRY, build_backbone
from .box_regression import Box2BoxTransform
from .meta_arch import META_ARCH_REGISTRY, GeneralizedRCNN, ProposalNetwork, SingleStageDetector, build_model
from .necks import FPN, NECK_REGISTRY, build_neck
from .poolers import ROIPooler, assign_boxes_to_levels
from .proposal_generator import PROPOSAL_GENERATOR_REGISTRY, RPN, RPN_HEAD_REGISTRY
from .roi_heads import ROI_BOX_HEAD_REGISTRY, ROI_HEADS_REGISTRY, ROI_MASK_HEAD_REGISTRY, StandardROIHeads
from .single_stage_heads import SINGLE_STAGE_HEADS_REGISTRY, RetinaNetHead
