"""Load converted weights into a model by reference variable name.

``read_tensor_file`` reads a flat {name: array} dict from .npz (no pickle),
.safetensors, or a torch .pth/.pt file through ``torch.load(weights_only=True)``
(a detectron2 training checkpoint keeps the state dict under "model").
detectron2's model-zoo .pkl files are pickles and are not opened here:
re-save them as .npz / .pth first.
"""
import os

import numpy as np
import torch

from .convert_d2 import convert_weights


def read_tensor_file(path):
    ext = os.path.splitext(path)[1].lower()
    if ext == ".npz":
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    if ext == ".safetensors":
        from safetensors.numpy import load_file
        return dict(load_file(path))
    if ext in (".pth", ".pt"):
        obj = torch.load(path, map_location="cpu", weights_only=True)
        if isinstance(obj, dict) and "model" in obj and isinstance(obj["model"], dict):
            obj = obj["model"]
        return {k: (v.numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in obj.items()}
    raise ValueError(f"unsupported checkpoint format {ext!r} (use .npz, .safetensors, .pth)")


OPTIONAL_STATE = ("loss_normalizer",)


def _optional_state(name):
    return name.rsplit("/", 1)[-1] in OPTIONAL_STATE


@torch.no_grad()
def load_reference_weights(model, tensors, strict=True):
    """Copy {reference variable name: array} into the model's parameters and
    buffers (Layer.reference_variables names, e.g. backbone/res2/block_1/conv1/
    norm/gamma).  Returns (missing, unexpected) name lists; strict raises on
    either, and on any shape mismatch."""
    own = dict(model.reference_variables(include_scope=False))
    # training-only state no detectron2 checkpoint carries (the RetinaNet
    # loss-normaliser EMA): optional, keeps its initial value when absent
    missing = [k for k in own if k not in tensors and not _optional_state(k)]
    unexpected = [k for k in tensors if k not in own]
    if strict and (missing or unexpected):
        raise KeyError(f"missing {missing[:5]}... ({len(missing)}), "
                       f"unexpected {unexpected[:5]}... ({len(unexpected)})")
    for k, t in own.items():
        if k not in tensors:
            continue
        v = torch.as_tensor(np.asarray(tensors[k]))
        if tuple(v.shape) != tuple(t.shape):
            raise ValueError(f"{k}: checkpoint shape {tuple(v.shape)} != model {tuple(t.shape)}")
        t.copy_(v.to(t.dtype))
    return missing, unexpected


def load_detectron2_checkpoint(model, path_or_dict, cfg, strict=True):
    """detectron2 weights (file or {name: array}) -> convert_weights
    (lib/convert_models/convert_d2.py) -> the model."""
    d = read_tensor_file(path_or_dict) if isinstance(path_or_dict, str) else dict(path_or_dict)
    tensors = convert_weights(d, cfg)
    # The reference converter names the RetinaNet tower "head/<conv>"
    # (convert_d2.py:77-81), its model scopes it "head/head/<conv>" (the
    # detector's "head" scope around RetinaNetHead's "head", retinanet.py:83,
    # single_stage_detector.py:26): a converted name the model lacks is looked
    # up under the tower scope too.
    own = {k for k, _ in model.reference_variables(include_scope=False)}
    tensors = {(("head/" + k) if k not in own and k.startswith("head/") and "head/" + k in own
                else k): v for k, v in tensors.items()}
    return load_reference_weights(model, tensors, strict=strict)
