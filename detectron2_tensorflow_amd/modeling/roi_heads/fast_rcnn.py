"""FastRCNNOutputLayers + inference (lib/modeling/roi_heads/fast_rcnn.py:28-435).

Inference (softmax, class-specific decode, clip, score threshold in the
class-major tf.where order, class-offset NMS with max_coord + 1, top-k and
padding) is the fused HIP pipeline d2mi_fast_rcnn_inference."""
import numpy as np

from ...layers import Layer, Linear
from ...layers import initializers as init
from ...layers import ops
from ...layers.loss import smooth_l1_loss

# GPU training takes the fused HIP losses (csrc/roi_losses.hip); False runs
# the tensor formulation below on the GPU too (tests compare the two).
FUSED_LOSSES = True


class FastRCNNOutputLayers(Layer):
    def __init__(self, input_size, num_classes, cls_agnostic_bbox_reg, box_dim=4, **kwargs):
        super().__init__(**kwargs)
        if not isinstance(input_size, int):
            input_size = int(np.prod(input_size))
        self.num_classes = num_classes
        self.cls_agnostic_bbox_reg = cls_agnostic_bbox_reg
        self.cls_score = Linear(input_size, num_classes + 1,
                                weights_initializer=init.random_normal(0.01), scope="class_logits")
        nreg = 1 if cls_agnostic_bbox_reg else num_classes
        self.bbox_pred = Linear(input_size, nreg * box_dim,
                                weights_initializer=init.random_normal(0.001), scope="box_deltas")

    def call(self, x):
        if x.dim() > 2:
            x = x.reshape(x.shape[0], -1)
        return self.cls_score(x), self.bbox_pred(x)


def fast_rcnn_inference(pred_class_logits, pred_proposal_deltas, proposal_boxes, roi_img, roi_slot,
                        num_images, num_slots, image_shapes, box2box_transform, score_thresh,
                        nms_thresh, topk_per_image, nms_cls_agnostic=False):
    """Returns (boxes [N,k,4], scores [N,k], classes int64 [N,k], is_valid [N,k],
    kept ROI row [N,k] (-1 pad)); rows with roi_slot < 0 are ignored.
    nms_cls_agnostic: one plain NMS over every class's filtered boxes
    (fast_rcnn.py:138-139) instead of the class-offset NMS."""
    K = pred_class_logits.shape[1] - 1
    agnostic = pred_proposal_deltas.shape[1] == 4 and K != 1
    return ops.fast_rcnn_inference(pred_class_logits, pred_proposal_deltas, proposal_boxes, roi_img,
                                   roi_slot, num_images, num_slots, image_shapes,
                                   box2box_transform.weights, score_thresh, nms_thresh,
                                   topk_per_image, cls_agnostic=agnostic,
                                   scale_clamp=box2box_transform.scale_clamp,
                                   nms_cls_agnostic=nms_cls_agnostic)


def fast_rcnn_losses(pred_class_logits, pred_proposal_deltas, proposal_boxes, gt_classes,
                     gt_boxes, valid, box2box_transform, smooth_l1_beta):
    """FastRCNNOutputs.losses on dense rows (fast_rcnn.py:269-357).

    Rows with ``valid`` False are the padding of the fixed [N * BATCH_SIZE_PER_IMAGE]
    layout and take no part (the reference drops them with SparseBoxList).
    loss_cls = mean softmax CE over the R valid rows; loss_box_reg = smooth-L1 of
    the gt-class deltas of foreground rows, summed, / R.  Both 0 when R == 0."""
    import torch
    if pred_class_logits.is_cuda and FUSED_LOSSES:
        lc, lb = ops.fast_rcnn_loss(pred_class_logits, pred_proposal_deltas, proposal_boxes,
                                    gt_classes, gt_boxes, valid, box2box_transform.weights,
                                    smooth_l1_beta)
        return {"loss_cls": lc, "loss_box_reg": lb}
    K = pred_class_logits.shape[1] - 1
    R = valid.sum().clamp(min=1).to(pred_class_logits.dtype)
    cls = torch.where(valid, gt_classes, torch.zeros_like(gt_classes)).long()
    ce = torch.nn.functional.cross_entropy(pred_class_logits, cls, reduction="none")
    loss_cls = torch.where(valid, ce, torch.zeros_like(ce)).sum() / R
    fg = valid & (gt_classes >= 0) & (gt_classes < K)
    nreg = pred_proposal_deltas.shape[1] // 4
    pred = pred_proposal_deltas.reshape(-1, nreg, 4)
    col = torch.zeros_like(cls) if nreg == 1 else torch.where(fg, cls, torch.zeros_like(cls))
    pred = torch.gather(pred, 1, col[:, None, None].expand(-1, 1, 4))[:, 0]
    target = box2box_transform.get_deltas(proposal_boxes, gt_boxes)
    target = torch.where(fg[:, None], target, torch.zeros_like(target))
    l1 = smooth_l1_loss(labels=target, predictions=pred, beta=smooth_l1_beta)
    loss_box = torch.where(fg[:, None], l1, torch.zeros_like(l1)).sum() / R
    return {"loss_cls": loss_cls, "loss_box_reg": loss_box}
