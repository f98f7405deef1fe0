"""get_activation (lib/layers/activation.py:10-20)."""
import torch
import torch.nn.functional as F


def _mish(x):
    return x * torch.tanh(F.softplus(x))


_ACTS = {
    "relu": torch.relu, "relu6": F.relu6, "sigmoid": torch.sigmoid, "tanh": torch.tanh,
    "leaky_relu": lambda x: F.leaky_relu(x, 0.1), "swish": F.silu, "mish": _mish,
}


def get_activation(activation):
    if activation is None or activation == "":
        return None
    if callable(activation):
        return activation
    if activation not in _ACTS:
        raise ValueError(f"{activation} is not recognized!")
    return _ACTS[activation]


def is_relu(fn):
    return fn is torch.relu or fn is F.relu or fn is torch.nn.functional.relu
