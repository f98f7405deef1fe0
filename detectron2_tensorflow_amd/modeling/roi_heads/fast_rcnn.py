"""FastRCNNOutputLayers + inference (lib/modeling/roi_heads/fast_rcnn.py:28-435).

Inference (softmax, class-specific decode, clip, score threshold in the
class-major tf.where order, class-offset NMS with max_coord + 1, top-k and
padding) is the fused HIP pipeline d2mi_fast_rcnn_inference."""
import numpy as np

from ...layers import Layer, Linear
from ...layers import initializers as init
from ...layers import ops


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
    kept ROI row [N,k] (-1 pad)); rows with roi_slot < 0 are ignored."""
    if nms_cls_agnostic:
        raise NotImplementedError("class-agnostic NMS is not on the hot path")
    K = pred_class_logits.shape[1] - 1
    agnostic = pred_proposal_deltas.shape[1] == 4 and K != 1
    return ops.fast_rcnn_inference(pred_class_logits, pred_proposal_deltas, proposal_boxes, roi_img,
                                   roi_slot, num_images, num_slots, image_shapes,
                                   box2box_transform.weights, score_thresh, nms_thresh,
                                   topk_per_image, cls_agnostic=agnostic,
                                   scale_clamp=box2box_transform.scale_clamp)
