"""SINGLE_STAGE_HEADS_REGISTRY (lib/modeling/single_stage_heads/build.py)."""
from ...utils.registry import Registry

SINGLE_STAGE_HEADS_REGISTRY = Registry("SINGLE_STAGE_HEADS")


def build_single_stage_head(cfg, input_shape, **kwargs):
    return SINGLE_STAGE_HEADS_REGISTRY.get(cfg.MODEL.SINGLE_STAGE_HEAD.NAME)(cfg, input_shape, **kwargs)
