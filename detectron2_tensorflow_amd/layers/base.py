"""Layer contract of the reference (lib/layers/base.py:11-63) on torch.nn.Module.

A Layer stores its constructor keywords as attributes, builds its
parameters in the constructor, and ``__call__`` runs ``call(...)``.
Parameters keep the reference variable names ("weights", "bias", "gamma",
"beta", "moving_mean", "moving_variance") and submodules are registered
under their reference scope names, so ``reference_variables()`` yields the
TF-style paths (e.g. ``neck/fpn_lateral2/weights``) a converted checkpoint
uses.
"""
import torch

from ..utils import training as _training


class Layer(torch.nn.Module):
    def __init__(self, dtype=torch.float32, scope=None, **kwargs):
        super().__init__()
        object.__setattr__(self, "layer_dtype", dtype)
        object.__setattr__(self, "scope", scope if scope is not None else type(self).__name__)
        training = kwargs.pop("training", None)
        for name, value in kwargs.items():
            if isinstance(value, torch.nn.Module):
                self.add_module(name, value)
            else:
                object.__setattr__(self, name, value)
        if training is None:
            try:
                training = _training.get_training_phase()
            except ValueError:
                training = False  # the reference raises here; inference is the safe default
        self.train(bool(training))

    def forward(self, *args, **kwargs):
        return self.call(*args, **kwargs)

    def call(self, *args, **kwargs):  # pragma: no cover - abstract
        raise NotImplementedError

    def add_layer(self, layer, name=None):
        """Register a child Layer under its reference scope name."""
        self.add_module(name or layer.scope, layer)
        return layer

    def reference_variables(self, prefix="", include_scope=True):
        """(reference variable path, tensor) pairs, e.g. ("neck/fpn_output2/weights", w).
        Layers inside ModuleLists are named by their own scopes (res2/block_1,
        mask_fcn1, fpn_lateral2 ...), as the reference's variable scopes;
        include_scope=False leaves out this layer's own scope (the meta-arch
        root: the reference's variables start at backbone/, neck/, ...)."""
        base = prefix + (self.scope + "/" if include_scope and self.scope else "")
        transient = getattr(self, "_non_persistent_buffers_set", set())
        bufs = [(n, b) for n, b in self.named_buffers(recurse=False) if n not in transient]
        for name, p in list(self.named_parameters(recurse=False)) + bufs:
            yield base + name, p

        def walk(mod, path):
            for name, child in mod.named_children():
                if isinstance(child, Layer):
                    yield from child.reference_variables(path)
                elif isinstance(child, (torch.nn.ModuleList, torch.nn.Sequential)):
                    yield from walk(child, path)
                else:
                    for pn, p in child.named_parameters():
                        yield path + name + "/" + pn.replace(".", "/"), p

        yield from walk(self, base)


class Sequential:
    """lib/layers/base.py:44-63."""

    def __init__(self, layers=None):
        layers = list(layers or [])
        for layer in layers:
            assert isinstance(layer, Layer)
        self._layers = layers

    def add(self, layer):
        assert isinstance(layer, Layer)
        self._layers.append(layer)

    def __call__(self, inputs):
        ret = inputs
        for layer in self._layers:
            ret = layer(ret)
        return ret
