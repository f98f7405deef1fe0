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

    def reference_variables(self, prefix=""):
        """(reference variable path, tensor) pairs, e.g. ("neck/fpn_output2/weights", w)."""
        base = prefix + (self.scope + "/" if prefix or self.scope else "")
        for name, p in list(self.named_parameters(recurse=False)) + list(self.named_buffers(recurse=False)):
            yield base + name, p
        for child in self.children():
            if isinstance(child, Layer):
                yield from child.reference_variables(base)
            else:
                for name, p in child.named_parameters():
                    yield base + name.replace(".", "/"), p


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
