from .build import PROPOSAL_GENERATOR_REGISTRY, build_proposal_generator
from .rpn import RPN, RPN_HEAD_REGISTRY, StandardRPNHead, build_rpn_head

__all__ = ["PROPOSAL_GENERATOR_REGISTRY", "build_proposal_generator", "RPN", "RPN_HEAD_REGISTRY",
           "StandardRPNHead", "build_rpn_head"]
