"""FastRCNNConvFCHead (lib/modeling/roi_heads/box_head.py:17-89).

The pooled [R, 7, 7, 256] NHWC features flatten in HWC order (the reference's
fc1 row order, convert_d2.py:153-162) and go through NUM_FC Linear + ReLU
(library GEMMs); optional NUM_CONV 3x3 convs run on the MFMA conv kernel."""
import numpy as np
import torch

from ...layers import Conv2D, Layer, Linear, get_norm
from ...layers import initializers as init
from ...utils.arg_scope import arg_scope
from ...utils.registry import Registry

ROI_BOX_HEAD_REGISTRY = Registry("ROI_BOX_HEAD")


@ROI_BOX_HEAD_REGISTRY.register()
class FastRCNNConvFCHead(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        h = cfg.MODEL.ROI_BOX_HEAD
        assert h.NUM_CONV + h.NUM_FC > 0
        self._output_size = (input_shape.channels, input_shape.height, input_shape.width)
        normalizer = get_norm(h.NORM)
        convs = []
        with arg_scope([Conv2D], out_channels=h.CONV_DIM, kernel_size=3, use_bias=not normalizer,
                       normalizer=normalizer, normalizer_params={"channels": h.CONV_DIM, "scope": "norm"},
                       activation="relu", padding="SAME",
                       weights_initializer=init.variance_scaling(2.0, mode="fan_out",
                                                                 distribution="untruncated_normal")):
            for k in range(h.NUM_CONV):
                convs.append(Conv2D(in_channels=self._output_size[0], scope=f"conv{k + 1}"))
                self._output_size = (h.CONV_DIM, self._output_size[1], self._output_size[2])
        self.convs = torch.nn.ModuleList(convs)
        fcs = []
        with arg_scope([Linear], out_units=h.FC_DIM, activation="relu",
                       weights_initializer=init.variance_scaling()):
            for k in range(h.NUM_FC):
                fcs.append(Linear(int(np.prod(self._output_size)), scope=f"fc{k + 1}"))
                self._output_size = h.FC_DIM
        self.fcs = torch.nn.ModuleList(fcs)

    def call(self, x):
        for layer in self.convs:
            x = layer(x)
        if len(self.fcs):
            if x.dim() > 2:
                x = x.reshape(x.shape[0], -1)
            for layer in self.fcs:
                x = layer(x)
        return x

    @property
    def output_size(self):
        return self._output_size


def build_box_head(cfg, input_shape, **kwargs):
    return ROI_BOX_HEAD_REGISTRY.get(cfg.MODEL.ROI_BOX_HEAD.NAME)(cfg, input_shape, **kwargs)
