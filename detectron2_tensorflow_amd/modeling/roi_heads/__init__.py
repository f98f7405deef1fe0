from .box_head import ROI_BOX_HEAD_REGISTRY, FastRCNNConvFCHead, build_box_head
from .fast_rcnn import FastRCNNOutputLayers
from .mask_head import ROI_MASK_HEAD_REGISTRY, MaskRCNNConvUpsampleHead, build_mask_head, mask_rcnn_inference
from .roi_heads import ROI_HEADS_REGISTRY, ROIHeads, StandardROIHeads, build_roi_heads

__all__ = ["ROI_BOX_HEAD_REGISTRY", "FastRCNNConvFCHead", "build_box_head", "FastRCNNOutputLayers",
           "ROI_MASK_HEAD_REGISTRY", "MaskRCNNConvUpsampleHead", "build_mask_head",
           "mask_rcnn_inference", "ROI_HEADS_REGISTRY", "ROIHeads", "StandardROIHeads",
           "build_roi_heads"]
