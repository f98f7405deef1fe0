"""MaskRCNNConvUpsampleHead + mask_rcnn_inference (lib/modeling/roi_heads/mask_head.py:71-180).

NUM_CONV 3x3 convs + ReLU, the 2x2/s2 transposed conv + ReLU (as one GEMM on
the MFMA kernel + pixel shuffle) and the 1x1 predictor, all on gfx950 MFMA."""
import torch

from ...layers import Conv2D, ConvTranspose2D, Layer, get_norm
from ...layers import initializers as init
from ...utils.arg_scope import arg_scope
from ...utils.registry import Registry

ROI_MASK_HEAD_REGISTRY = Registry("ROI_MASK_HEAD")


def mask_rcnn_inference(pred_mask_logits, pred_classes):
    """[B, Hm, Wm, C] logits -> sigmoid of the predicted class's channel
    (class-agnostic: channel 0; the reference's channel-1 gather at
    mask_head.py:98 is a bug not reproduced)."""
    B = pred_mask_logits.shape[0]
    if pred_mask_logits.shape[-1] == 1:
        logits = pred_mask_logits[..., 0]
    else:
        idx = pred_classes.reshape(B).clamp(min=0).to(torch.int64)
        logits = pred_mask_logits[torch.arange(B, device=idx.device), :, :, idx]
    return torch.sigmoid(logits)


@ROI_MASK_HEAD_REGISTRY.register()
class MaskRCNNConvUpsampleHead(Layer):
    def __init__(self, cfg, input_shape, **kwargs):
        super().__init__(**kwargs)
        num_classes = cfg.MODEL.ROI_HEADS.NUM_CLASSES
        m = cfg.MODEL.ROI_MASK_HEAD
        normalizer = get_norm(m.NORM)
        convs = []
        with arg_scope([Conv2D, ConvTranspose2D],
                       weights_initializer=init.variance_scaling(2.0, mode="fan_out",
                                                                 distribution="untruncated_normal"),
                       activation="relu"):
            for k in range(m.NUM_CONV):
                convs.append(Conv2D(input_shape.channels if k == 0 else m.CONV_DIM, m.CONV_DIM, 3,
                                    use_bias=not normalizer, normalizer=normalizer,
                                    normalizer_params={"channels": m.CONV_DIM, "scope": "norm"},
                                    padding="SAME", scope=f"mask_fcn{k + 1}"))
            self.convs = torch.nn.ModuleList(convs)
            self.deconv = ConvTranspose2D(m.CONV_DIM if m.NUM_CONV > 0 else input_shape.channels,
                                          m.CONV_DIM, kernel_size=2, stride=2, scope="deconv")
            nmask = 1 if m.CLS_AGNOSTIC_MASK else num_classes
            self.predictor = Conv2D(m.CONV_DIM, nmask, 1, activation=None,
                                    weights_initializer=init.random_normal(0.001), scope="predictor")

    def call(self, x):
        for layer in self.convs:
            x = layer(x)
        deconv = self.deconv(x)
        return deconv, self.predictor(deconv)


def build_mask_head(cfg, input_shape, **kwargs):
    return ROI_MASK_HEAD_REGISTRY.get(cfg.MODEL.ROI_MASK_HEAD.NAME)(cfg, input_shape, **kwargs)
