"""Functional ops of lib/layers/functional.py (:1-187), NHWC.

``crop_and_resize`` (:100-166) is the reference's ROIAlign math; here it is one
launch of the HIP kernel d2mi_roi_align_fwd (the SYMMETRIC pad is folded into
the kernel's index clamp, so no padded copy of the map is made).
"""
import torch
import torch.nn.functional as F

from . import ops


def resize_images(images, size, method="bilinear", **kwargs):
    """resize_images (:9-36) on NHWC.  With TF >= 1.14 the reference takes the
    tf.compat.v2.image.resize branch, whose kwargs filter drops align_corners:
    bilinear is ResizeBilinear with half-pixel centres and no antialias, run
    here by the HIP kernel (d2mi_resize_bilinear, TF 1.15 arithmetic; GPU
    tensors only).  Other methods are not on the hot path: PyTorch's
    interpolate (half-pixel for bicubic / area; nearest is floor-indexed)."""
    x = images if images.dim() == 4 else images[None]
    if method == "bilinear":
        y = ops.resize_bilinear_grad(x, size)
    else:
        mode = {"nearest": "nearest", "bicubic": "bicubic", "area": "area"}[method]
        kw = {"align_corners": False} if mode == "bicubic" else {}
        y = F.interpolate(x.permute(0, 3, 1, 2), size=tuple(int(s) for s in size), mode=mode,
                          **kw).permute(0, 2, 3, 1)
    return y if images.dim() == 4 else y[0]


def subsample(inputs, factor, scope=None):
    """max_pool2d [1,1] stride factor == strided slice (:36-55)."""
    return inputs if factor == 1 else inputs[:, ::factor, ::factor, :]


def upsample(inputs, factor, scope=None):
    """Nearest x factor (:58-90): out[i] = in[i // factor]."""
    if factor == 1:
        return inputs
    return inputs.repeat_interleave(factor, dim=1).repeat_interleave(factor, dim=2)


def flatten(inputs, scope=None):
    return inputs if inputs.dim() <= 2 else inputs.reshape(inputs.shape[0], -1)


def crop_and_resize(image, boxes, box_ind, crop_size, aligned=True, method="bilinear",
                    pad_border=True):
    """Aligned crop_and_resize on fp-coordinate boxes [n, 4] (ymin, xmin, ymax, xmax)."""
    if method != "bilinear":
        raise NotImplementedError("only bilinear crop_and_resize is on the hot path")
    return ops.roi_align([image], boxes.detach(), box_ind, tuple(crop_size), [1.0], 0,
                         aligned=aligned, pad_border=pad_border)


def tf_crop_and_resize(image, boxes, box_ind, crop_size):
    """tf.image.crop_and_resize on normalised boxes (used by the mask loss,
    mask_head.py:51, and mask pasting, mask_ops.py:50)."""
    return ops.roi_align([image], boxes, box_ind, tuple(crop_size), [1.0], 0, pad_border=False,
                         box_mode=ops.BOX_MODE_RAW)


def drop_connect(inputs, is_training, drop_connect_rate):
    if not is_training or not drop_connect_rate:
        return inputs
    keep = 1.0 - drop_connect_rate
    mask = torch.floor(keep + torch.rand(inputs.shape[0], 1, 1, 1, device=inputs.device))
    return inputs / keep * mask
