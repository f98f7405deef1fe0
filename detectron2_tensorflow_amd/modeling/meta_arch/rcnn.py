"""GeneralizedRCNN / ProposalNetwork (lib/modeling/meta_arch/rcnn.py:17-224).

batched_inputs is the reference's dict: "image" [N, H, W, 3] float32 0-255
RGB (NHWC), "image_shape" [N, 2] int32 true (h, w).  Preprocessing
normalises, THEN flips to BGR when INPUT_FORMAT == "BGR", then zero-pads to
the neck's size divisibility (rcnn.py:146-157, image_list.py:89-100).
Inference returns {"instances": {boxes, classes, scores, is_valid[, masks]}}
as dense [N, DETECTIONS_PER_IMAGE] tensors (fields.ResultFields names); masks
are the 28x28 probabilities ("raw") or uint8 masks pasted onto the canvas
("conventional" / "fixed", modeling/postprocessing.py).

Training (rcnn.py:62-90) takes batched_inputs["instances"] as a dict of dense
padded ground truth: gt_boxes [N, G, 4] (y1, x1, y2, x2, absolute),
gt_classes [N, G] (0-based), is_valid [N, G], optional gt_is_crowd /
gt_difficult [N, G] and gt_masks [N, G, 56, 56] mini masks (MASK_ON), and
returns the dict of scalar losses.
"""
import torch

from ...layers import Layer
from ...structures import ImageList
from ..backbone import build_backbone
from ..necks import build_neck
from ..proposal_generator import build_proposal_generator
from ..postprocessing import detector_postprocess
from ..roi_heads import build_roi_heads
from .build import META_ARCH_REGISTRY


class _Preprocess:
    def _init_preprocess(self, cfg):
        assert len(cfg.MODEL.PIXEL_MEAN) == len(cfg.MODEL.PIXEL_STD)
        self.register_buffer("pixel_mean", torch.tensor(cfg.MODEL.PIXEL_MEAN, dtype=torch.float32),
                             persistent=False)
        self.register_buffer("pixel_std", torch.tensor(cfg.MODEL.PIXEL_STD, dtype=torch.float32),
                             persistent=False)
        self.input_format = cfg.MODEL.INPUT_FORMAT

    def preprocess_image(self, batched_inputs):
        from ...layers import ops
        x = batched_inputs["image"]
        if x.is_cuda and ops.FUSED_PREPROCESS and x.dim() == 4 and x.shape[-1] == 3:
            # one launch: normalise, flip, pad (d2mi_preprocess_images)
            images = ops.preprocess_images(x, self.pixel_mean, self.pixel_std,
                                           self.input_format == "BGR", self.neck.size_divisibility)
            shapes = batched_inputs["image_shape"].to(device=images.device, dtype=torch.int32)
            return ImageList.from_tensors(images, shapes, 0)
        images = (x - self.pixel_mean) / self.pixel_std
        if self.input_format == "BGR":
            images = images.flip(-1)
        shapes = batched_inputs["image_shape"].to(device=images.device, dtype=torch.int32)
        return ImageList.from_tensors(images.contiguous(), shapes, self.neck.size_divisibility)


@META_ARCH_REGISTRY.register()
class GeneralizedRCNN(_Preprocess, Layer):
    def __init__(self, cfg, **kwargs):
        super().__init__(**kwargs)
        self.backbone = build_backbone(cfg, scope="backbone")
        self.neck = build_neck(cfg, self.backbone.output_shape(), scope="neck")
        self.proposal_generator = build_proposal_generator(cfg, self.neck.output_shape(),
                                                           scope="proposal_generator")
        self.roi_heads = build_roi_heads(cfg, self.neck.output_shape(), scope="roi_heads")
        self._init_preprocess(cfg)
        self.segmentation_output_format = cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT
        self.segmentation_output_resolution = cfg.MODEL.SEGMENTATION_OUTPUT.FIXED_RESOLUTION

    def _tag_shared_levels(self, features):
        """FPN levels read by both the RPN head conv and the ROI poolers get a
        gradient hand-off dict (the pair_grad protocol): whichever backward
        runs first leaves its input gradient there and the other adds into it
        (the RPN dgrad epilogue, or the merged ROIAlign backward accumulating
        at touched pixels) -- no autograd add of two full maps, no zero-fill
        of the pooled levels.  Only when the ROI heads take the merged
        backward (box + mask poolers), which always consumes the hand-off."""
        from ...layers import ops
        rh, pg = self.roi_heads, self.proposal_generator
        if (pg is None or not getattr(rh, "mask_on", False) or not ops.MERGED_BWD
                or not hasattr(pg, "rpn_head")):
            return
        shared = set(rh.in_features) & set(getattr(pg, "in_features", ()))
        for f in shared:
            t = features[f]
            if t.is_cuda and t.requires_grad and t.shape[-1] >= 64:
                t._d2mi_grad_pair = {}

    def call(self, batched_inputs):
        if not self.training:
            return self.inference(batched_inputs)
        images = self.preprocess_image(batched_inputs)
        gt = batched_inputs.get("instances", batched_inputs.get("targets"))
        features = self.neck(self.backbone(images.tensor))
        self._tag_shared_levels(features)
        if self.proposal_generator is not None:
            proposals, proposal_losses, _ = self.proposal_generator(images, features, gt)
        else:
            proposals, proposal_losses = batched_inputs["proposals"], {}
        _, detector_losses = self.roi_heads(images, features, proposals, gt)
        losses = {}
        losses.update(detector_losses)
        losses.update(proposal_losses)
        return losses

    def inference(self, batched_inputs, detected_instances=None):
        assert not self.training
        images = self.preprocess_image(batched_inputs)
        features = self.neck(self.backbone(images.tensor))
        if detected_instances is None:
            if self.proposal_generator is not None:
                proposals, *_ = self.proposal_generator(images, features, None)
            else:
                proposals = batched_inputs["proposals"]
            results, _ = self.roi_heads(images, features, proposals, None)
        else:
            results = self.roi_heads.forward_with_given_boxes(features, detected_instances)
        out = {"boxes": results.boxes, "classes": results.get_field("pred_classes"),
               "scores": results.get_field("scores"), "is_valid": results.get_field("is_valid")}
        if results.has_field("pred_masks"):
            out["masks"] = results.get_field("pred_masks")
            fmt = self.segmentation_output_format
            if fmt != "raw":  # rcnn.py:124-133
                if fmt == "fixed":
                    shape = (self.segmentation_output_resolution,) * 2
                else:  # "conventional": the padded input canvas
                    shape = tuple(images.tensor.shape[1:3])
                out = detector_postprocess(out, shape, fmt, images.image_shapes)
        return {"instances": out}


@META_ARCH_REGISTRY.register()
class ProposalNetwork(_Preprocess, Layer):
    """rcnn.py:161-224: backbone + neck + RPN, returns the proposals."""

    def __init__(self, cfg, **kwargs):
        super().__init__(**kwargs)
        self.backbone = build_backbone(cfg, scope="backbone")
        self.neck = build_neck(cfg, self.backbone.output_shape(), scope="neck")
        self.proposal_generator = build_proposal_generator(cfg, self.neck.output_shape(),
                                                           scope="proposal_generator")
        self._init_preprocess(cfg)

    def call(self, batched_inputs):
        images = self.preprocess_image(batched_inputs)
        features = self.neck(self.backbone(images.tensor))
        gt = batched_inputs.get("instances") if self.training else None
        proposals, losses, _ = self.proposal_generator(images, features, gt)
        if self.training:
            return losses
        return {"proposals": {"boxes": proposals.boxes,
                              "objectness_logits": proposals.get_field("objectness_logits"),
                              "is_valid": proposals.get_field("is_valid")}}
