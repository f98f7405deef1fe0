"""SingleStageDetector (lib/modeling/meta_arch/single_stage_detector.py:16-83)."""
from ...layers import Layer
from ..backbone import build_backbone
from ..necks import build_neck
from ..single_stage_heads import build_single_stage_head
from .build import META_ARCH_REGISTRY
from .rcnn import _Preprocess


@META_ARCH_REGISTRY.register()
class SingleStageDetector(_Preprocess, Layer):
    def __init__(self, cfg, **kwargs):
        super().__init__(**kwargs)
        self.backbone = build_backbone(cfg, scope="backbone")
        self.neck = build_neck(cfg, self.backbone.output_shape(), scope="neck")
        self.detector = build_single_stage_head(cfg, self.neck.output_shape(), scope="head")
        self._init_preprocess(cfg)

    def call(self, batched_inputs):
        images = self.preprocess_image(batched_inputs)
        features = self.neck(self.backbone(images.tensor))
        gt = batched_inputs.get("instances")
        results, losses = self.detector(images, features, gt)
        if self.training:
            return losses
        out = {"boxes": results.boxes, "classes": results.get_field("pred_classes"),
               "scores": results.get_field("scores"), "is_valid": results.get_field("is_valid")}
        if results.has_field("pred_masks"):  # single_stage_detector.py:75-76 (SOLOv2)
            out["masks"] = results.get_field("pred_masks")
        return {"instances": out}
