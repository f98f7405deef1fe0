"""ROIAlign layer (lib/layers/roi_align.py:9-75) on the gfx950 ROIAlign kernel."""
from . import ops
from .base import Layer


class ROIAlign(Layer):
    def __init__(self, output_size, spatial_scale, sampling_ratio, aligned=True):
        """output_size (h, w); boxes are scaled by spatial_scale; sampling_ratio
        > 0 crops at output*SR and averages SR x SR samples; aligned selects
        the ROIAlignV2 box transform (lib/layers/functional.py:138-152)."""
        assert isinstance(sampling_ratio, int), sampling_ratio
        super().__init__(output_size=tuple(output_size), spatial_scale=spatial_scale,
                         sampling_ratio=sampling_ratio, aligned=aligned)

    def call(self, inputs, boxes, box_inds):
        return ops.roi_align([inputs], boxes.detach(), box_inds, self.output_size,
                             [self.spatial_scale], self.sampling_ratio, aligned=self.aligned)

    def __repr__(self):
        return (f"ROIAlign(output_size={self.output_size}, spatial_scale={self.spatial_scale}, "
                f"sampling_ratio={self.sampling_ratio}, aligned={self.aligned})")
