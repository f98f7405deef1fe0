"""Synthetic COCO-shaped batches for bench / tests.

Images U[0, 255) at the padded-to-/32 size, and for training 7 GT boxes per
image with log-uniform sqrt(area) in [32, 512], log-uniform aspect ratio in
[0.5, 2], centres uniform inside the image (boxes clipped to it), classes
U{0..K-1}, and box-filled 56x56 mini masks (all ones, the shape
TRANSFORM.RESIZE.USE_MINI_MASKS produces).  Seeded; generated on the host
once and moved to the device, so the timed region reads it from HBM.
"""
import numpy as np
import torch


def synthetic_images(batch, height, width, seed, device):
    g = torch.Generator(device="cpu").manual_seed(seed)
    img = torch.rand(batch, height, width, 3, generator=g) * 255.0
    shapes = torch.tensor([[height, width]] * batch, dtype=torch.int32)
    return {"image": img.to(device), "image_shape": shapes.to(device)}


def synthetic_instances(batch, height, width, seed, device, num_gt=7, num_classes=80,
                        mask_size=56, sqrt_area=(32.0, 512.0), full_mask_hw=None):
    """full_mask_hw: (H, W) -- image-size box-filled masks [batch, num_gt, H, W]
    instead of the mini masks (SOLOv2 training: get_ground_truth takes the
    masks at the padded image size, solo_v2.py:399-401)."""
    rng = np.random.default_rng(seed)
    n = batch * num_gt
    s = np.exp(rng.uniform(np.log(sqrt_area[0]), np.log(sqrt_area[1]), n))
    r = np.exp(rng.uniform(np.log(0.5), np.log(2.0), n))  # h / w
    h, w = s * np.sqrt(r), s / np.sqrt(r)
    cy, cx = rng.uniform(0, height, n), rng.uniform(0, width, n)
    boxes = np.stack([np.clip(cy - h / 2, 0, height), np.clip(cx - w / 2, 0, width),
                      np.clip(cy + h / 2, 0, height), np.clip(cx + w / 2, 0, width)], 1)
    # keep every box at least 4 px on a side after clipping
    boxes[:, 2] = np.maximum(boxes[:, 2], boxes[:, 0] + 4)
    boxes[:, 3] = np.maximum(boxes[:, 3], boxes[:, 1] + 4)
    inst = {
        "gt_boxes": torch.from_numpy(boxes.astype(np.float32).reshape(batch, num_gt, 4)),
        "gt_classes": torch.from_numpy(rng.integers(0, num_classes, (batch, num_gt))),
        "is_valid": torch.ones(batch, num_gt, dtype=torch.bool),
        "gt_is_crowd": torch.zeros(batch, num_gt, dtype=torch.bool),
        "gt_difficult": torch.zeros(batch, num_gt, dtype=torch.bool),
        "gt_masks": torch.ones(batch, num_gt, mask_size, mask_size, dtype=torch.uint8),
    }
    if full_mask_hw is not None:
        H, W = full_mask_hw
        yy = torch.arange(H).view(1, 1, H, 1).float()
        xx = torch.arange(W).view(1, 1, 1, W).float()
        b = inst["gt_boxes"]
        # pixel (y, x) inside when its centre is: y + 0.5 in (y1, y2)
        inst["gt_masks"] = (((yy + 0.5) > b[..., 0, None, None]) & ((yy + 0.5) < b[..., 2, None, None])
                            & ((xx + 0.5) > b[..., 1, None, None])
                            & ((xx + 0.5) < b[..., 3, None, None])).to(torch.uint8)
    return {k: v.to(device) for k, v in inst.items()}


def synthetic_train_batch(batch, height, width, seed, device, **kw):
    out = synthetic_images(batch, height, width, seed, device)
    out["instances"] = synthetic_instances(batch, height, width, seed, device, **kw)
    return out


@torch.no_grad()
def calibrate_rcnn_scores(model, batch):
    """BASELINE.md score injection for a random-init (Mask / Faster) R-CNN:
    rescale the box-head class logits to ~ N(0, 3^2), the RPN objectness to
    ~ N(0, 1) and the RPN anchor deltas to N(0, 0.1^2) on this batch's
    features; also the box-head deltas to ~ N(0, 0.5^2) and the mask logits
    to ~ N(0, 1).  The unnormalised features of a random-init ResNet otherwise
    give class logits in the hundreds (a Fast R-CNN CE loss of ~750), deltas
    of O(10), which collapse most proposals onto the image border, and mask
    logits of O(10) (a saturated BCE of ~13 whose size depends on the image
    size) -- random-init artefacts, not a training distribution.  The
    rescaling changes weights only, never the work a step does."""
    import math
    stats = {}

    def grab(name):
        def hook(mod, inp, out):
            x = inp[0]
            stats[name] = float((x.reshape(-1, x.shape[-1]) ** 2).sum(-1).mean())
        return hook

    rh = model.roi_heads
    h1 = rh.box_predictor.register_forward_hook(grab("box"))
    rpn_head = model.proposal_generator.rpn_head
    # the shared conv's output on the last level (the head returns them all)
    h2 = rpn_head.register_forward_hook(lambda m, i, o: stats.__setitem__(
        "rpn", float((o[0][-1].reshape(-1, o[0][-1].shape[-1]) ** 2).sum(-1).mean())))
    mask_pred = getattr(getattr(rh, "mask_head", None), "predictor", None)
    h3 = mask_pred.register_forward_hook(grab("mask")) if mask_pred is not None else None
    was = model.training
    model.eval()
    model.inference({"image": batch["image"], "image_shape": batch["image_shape"]})
    model.train(was)
    h1.remove()
    h2.remove()
    if h3 is not None:
        h3.remove()
    cls = rh.box_predictor.cls_score
    cls.weights.normal_(0.0, 3.0 / math.sqrt(max(stats["box"], 1e-12)))
    obj = rpn_head.objectness_logits
    obj.weights.normal_(0.0, 1.0 / math.sqrt(max(stats["rpn"], 1e-12)))
    rpn_head.anchor_deltas.weights.normal_(0.0, 0.1 / math.sqrt(max(stats["rpn"], 1e-12)))
    rh.box_predictor.bbox_pred.weights.normal_(0.0, 0.5 / math.sqrt(max(stats["box"], 1e-12)))
    if "mask" in stats:
        mask_pred.weights.normal_(0.0, 1.0 / math.sqrt(max(stats["mask"], 1e-12)))


@torch.no_grad()
def calibrate_solo_head(branch, pred_cls, pred_kernels, cls_mean=-4.5, cls_std=1.0,
                        kernel_std=0.1):
    """Score injection for a random-init SOLOv2 MaskKernelBranch: rescale
    solo_cate so the category logits are ~ N(cls_mean, cls_std^2) (a few
    hundred to a few thousand (cell, class) candidates above
    SCORE_THRESH_TEST = 0.1 after point NMS) and solo_kernel so the dynamic
    kernels have std kernel_std (mask logits of O(1): masks neither empty nor
    full).  pred_cls / pred_kernels: the branch's outputs on the features the
    calibration is for."""
    def std_wo_bias(outs, bias):
        return float(torch.cat([(o - bias.to(o.device)).reshape(-1) for o in outs]).double().std())

    s = std_wo_bias(pred_cls, branch.solo_cate.bias)
    branch.solo_cate.weights.mul_(cls_std / max(s, 1e-12))
    branch.solo_cate.bias.fill_(cls_mean)
    s = std_wo_bias(pred_kernels, branch.solo_kernel.bias)
    branch.solo_kernel.weights.mul_(kernel_std / max(s, 1e-12))
    branch.solo_kernel.bias.zero_()


def calibrate_retinanet_head(tower, box_cls, box_delta, cls_mean=-3.0, cls_std=1.0,
                             delta_std=0.1):
    """BASELINE.md score injection for a random-init RetinaNet: rescale the
    cls_score / bbox_pred conv weights (the convs are linear in their weights)
    so that, on the features that produced ``box_cls`` / ``box_delta`` (the
    head's outputs, any device), the class logits are ~ N(cls_mean, cls_std^2)
    and the deltas ~ N(0, delta_std^2).  A random-init ResNet's unnormalised
    features otherwise give logits of std ~20 (every sigmoid saturates to 1.0)
    and deltas of O(10)."""
    def std_wo_bias(outs, bias):
        return float(torch.cat([(o - bias.to(o.device)).reshape(-1) for o in outs]).double().std())

    s = std_wo_bias(box_cls, tower.cls_score.bias)
    tower.cls_score.weights.mul_(cls_std / max(s, 1e-12))
    tower.cls_score.bias.fill_(cls_mean)
    s = std_wo_bias(box_delta, tower.bbox_pred.bias)
    tower.bbox_pred.weights.mul_(delta_std / max(s, 1e-12))
    tower.bbox_pred.bias.zero_()
