"""Op surface of the reference's lib/layers (lib/layers/__init__.py:1-11)."""
from .activation import get_activation
from .base import Layer, Sequential
from .convolutional import Conv2D, ConvTranspose2D, fix_padding
from .functional import (crop_and_resize, drop_connect, flatten, resize_images, subsample,
                         tf_crop_and_resize, upsample)
from .nms import batch_nms, matrix_nms
from .normalization import BatchNorm, GroupNorm, get_norm
from .roi_align import ROIAlign
from .shape_spec import ShapeSpec
from .wrappers import Linear, MaxPool2D, Upsample

__all__ = [
    "Layer", "Sequential", "Conv2D", "ConvTranspose2D", "fix_padding", "BatchNorm", "GroupNorm",
    "get_norm", "Linear", "Upsample", "MaxPool2D", "ROIAlign", "resize_images", "upsample",
    "subsample", "flatten", "crop_and_resize", "tf_crop_and_resize", "drop_connect", "batch_nms",
    "matrix_nms", "ShapeSpec", "get_activation",
]
