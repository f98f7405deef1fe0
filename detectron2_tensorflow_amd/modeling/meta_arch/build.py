"""META_ARCH_REGISTRY / build_model (lib/modeling/meta_arch/build.py:3-16)."""
from ...utils.registry import Registry

META_ARCH_REGISTRY = Registry("META_ARCH")


def build_model(cfg, **kwargs):
    return META_ARCH_REGISTRY.get(cfg.MODEL.META_ARCHITECTURE)(cfg, **kwargs)
