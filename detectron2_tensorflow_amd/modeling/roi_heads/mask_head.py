"""MaskRCNNConvUpsampleHead + mask_rcnn_inference (lib/modeling/roi_heads/mask_head.py:71-180).

NUM_CONV 3x3 convs + ReLU, the 2x2/s2 transposed conv + ReLU (as one GEMM on
the MFMA kernel + pixel shuffle) and the 1x1 predictor, all on gfx950 MFMA."""
import torch

from ...layers import Conv2D, ConvTranspose2D, Layer, get_norm
from ...layers import initializers as init
from ...layers import ops
from ...utils.arg_scope import arg_scope
from ...utils.registry import Registry

ROI_MASK_HEAD_REGISTRY = Registry("ROI_MASK_HEAD")

# GPU training takes the fused HIP loss (csrc/roi_losses.hip); False runs the
# tensor formulation on the GPU too (tests compare the two).
FUSED_LOSSES = True


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


def mask_rcnn_loss(pred_mask_logits, boxes, gt_boxes, gt_classes, gt_masks, mask_ind, fg,
                   use_mini_masks):
    """mask_head.py:17-68 on dense rows.

    pred_mask_logits [B, Hm, Wm, C]; boxes / gt_boxes [B, 4] (proposal, matched GT);
    gt_classes [B]; gt_masks [M, h, w] (mini masks when use_mini_masks); mask_ind [B]
    row of gt_masks per ROI; fg [B] rows that count (the foreground proposals).
    Targets: tf.image.crop_and_resize of the GT mask to Hm x Wm (ROI coordinates
    normalised to the GT box for mini masks), rounded; loss: mean sigmoid CE of the
    GT-class channel over fg rows x Hm x Wm (0 with no foreground)."""
    from ...layers.functional import tf_crop_and_resize
    B, Hm, Wm, C = pred_mask_logits.shape
    if use_mini_masks:
        # ((y1 - gy1) / gh, (x1 - gx1) / gw, (y2 - gy1) / gh, (x2 - gx1) / gw)
        # with gh = gy2 - gy1, gw = gx2 - gx1: the same f32 operations,
        # broadcast over the two corners (3 launches instead of 11)
        g0 = gt_boxes[:, None, :2]
        boxes = ((boxes.reshape(B, 2, 2) - g0) / (gt_boxes[:, None, 2:] - g0)).reshape(B, 4)
    masks = gt_masks.to(torch.float32)[..., None].contiguous()
    ind = torch.where(fg, mask_ind.to(torch.int32), 0)
    with torch.no_grad():
        target = tf_crop_and_resize(masks, boxes.detach().contiguous(), ind, (Hm, Wm))
        target = torch.round(target[..., 0])
    if pred_mask_logits.is_cuda and FUSED_LOSSES:
        return ops.mask_loss(pred_mask_logits, target, gt_classes, fg)
    if C == 1:
        logits = pred_mask_logits[..., 0]
    else:
        cls = torch.where(fg, gt_classes, torch.zeros_like(gt_classes)).clamp(0, C - 1).long()
        logits = torch.gather(pred_mask_logits, 3, cls[:, None, None, None].expand(B, Hm, Wm, 1))[..., 0]
    bce = torch.nn.functional.binary_cross_entropy_with_logits(logits, target, reduction="none")
    n = (fg.sum() * (Hm * Wm)).clamp(min=1).to(bce.dtype)
    return torch.where(fg[:, None, None], bce, torch.zeros_like(bce)).sum() / n


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
        # each conv (and the deconv) is the sole consumer of the previous ReLU
        # output: its dgrad applies that ReLU's mask
        for i, layer in enumerate(self.convs):
            x = layer(x, relu_input_sole_consumer=i > 0)
        deconv = self.deconv(x, relu_input_sole_consumer=len(self.convs) > 0)
        return deconv, self.predictor(deconv)


def build_mask_head(cfg, input_shape, **kwargs):
    return ROI_MASK_HEAD_REGISTRY.get(cfg.MODEL.ROI_MASK_HEAD.NAME)(cfg, input_shape, **kwargs)
