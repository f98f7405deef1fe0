"""detector_postprocess (lib/modeling/postprocessing.py:9-59) on the dense
inference outputs.

"conventional": every box mask is pasted onto the padded input canvas
(output_shape = the batched image tensor's H, W); "fixed": onto a
FIXED_RESOLUTION square, boxes first scaled by output_shape / image_shape
(float64 ratio cast to float32, as TF's int32 truediv + box_list_ops.scale).
Both run d2mi_paste_masks (crop_and_resize of the reverse box + tf.greater
fused, uint8 out).  Padded detection slots (is_valid False) come back as zero
masks, as SparseBoxList.to_dense leaves them.

"raw": the reference's branch reads an undefined name (postprocessing.py:54)
and GeneralizedRCNN never calls it for "raw" (rcnn.py:124); here it
thresholds the box masks to uint8, its evident intent.
"""
import torch

from ..layers import ops


def detector_postprocess(instances, output_shape, mask_format, image_shapes=None,
                         mask_threshold=0.5):
    """instances: dict of dense [N, D, ...] tensors (boxes, is_valid, masks
    [N, D, mh, mw] probabilities).  Returns the dict with masks replaced by
    uint8 masks ([N, D, H, W] for the pasted formats)."""
    if "masks" not in instances:
        return instances
    masks = instances["masks"]
    out = dict(instances)
    if mask_format in ("conventional", "fixed"):
        N, D, mh, mw = masks.shape
        H, W = int(output_shape[0]), int(output_shape[1])
        yx = None
        if mask_format == "fixed":
            assert image_shapes is not None, "Detection results should carry the true input shape."
            target = torch.tensor([H, W], dtype=torch.float64, device=masks.device)
            yx = (target[None, :] / image_shapes.to(masks.device, torch.float64)).to(torch.float32)
            yx = yx.repeat_interleave(D, dim=0)
        pasted = ops.paste_masks(masks.reshape(N * D, mh, mw), instances["boxes"].reshape(N * D, 4),
                                 (H, W), valid=instances["is_valid"].reshape(N * D),
                                 yx_scale=yx, threshold=mask_threshold)
        out["masks"] = pasted.reshape(N, D, H, W)
    elif mask_format == "raw":
        out["masks"] = (masks > mask_threshold).to(torch.uint8)
    else:
        raise ValueError(f"mask format '{mask_format}' is not recognized.")
    return out
