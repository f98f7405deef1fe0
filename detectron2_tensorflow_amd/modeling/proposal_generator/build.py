"""PROPOSAL_GENERATOR_REGISTRY (lib/modeling/proposal_generator/build.py)."""
from ...utils.registry import Registry

PROPOSAL_GENERATOR_REGISTRY = Registry("PROPOSAL_GENERATOR")


def build_proposal_generator(cfg, input_shape, **kwargs):
    name = cfg.MODEL.PROPOSAL_GENERATOR.NAME
    if name == "PrecomputedProposals":
        return None
    return PROPOSAL_GENERATOR_REGISTRY.get(name)(cfg, input_shape, **kwargs)
