"""META_ARCH_REGISTRY / build_model (lib/modeling/meta_arch/build.py:3-16)."""
from ...layers.convolutional import PackGroup
from ...utils.registry import Registry

META_ARCH_REGISTRY = Registry("META_ARCH")


def build_model(cfg, **kwargs):
    model = META_ARCH_REGISTRY.get(cfg.MODEL.META_ARCHITECTURE)(cfg, **kwargs)
    if PackGroup.ENABLED:
        PackGroup.attach(model)  # its un-normalised convs repack in one batch per step
    return model
