"""ORACLE — test infrastructure only.  CPU restatement of ONE Mask R-CNN R50-FPN
training iteration (lib/modeling/meta_arch/rcnn.py:62-90 under
lib/engine/trainer.py:116-139), used as bench.py's ``cpu_baseline`` for the
training workload.  Never imported by the product path.

  forward: the same torch-CPU convs / FrozenBN / FPN as cpu_pipeline.py, now
  with autograd; RPN losses by the package's device-agnostic loss code on
  oracle-generated anchors (rpn_outputs.py:306-401); proposals by the numpy /
  C restatement of find_top_rpn_proposals with the TRAIN top-k
  (rpn_outputs.py:29-132); ROI sampling and box / mask losses by the package's
  torch code (roi_heads.py:100-232, fast_rcnn.py:269-357, mask_head.py:17-68)
  with the mask targets from the C tf.image.crop_and_resize;
  ROIAlign forward = the C restatement (functional.py:100-166), backward =
  CropAndResizeGradImage in C on the SYMMETRIC-padded map + MirrorPadGrad fold;
  backward: torch-CPU autograd; update: per-tensor clip + Momentum-SGD.
"""
import copy

import numpy as np
import torch
import torch.nn.functional as F

import oracle
from cpu_pipeline import _backbone, _conv, _fpn

F32 = np.float32


def _aligned_boxes(boxes, scale, crop, H, W):
    """transform_fpcoor_for_tf, aligned, on the padded map (functional.py:122-149)."""
    b = boxes.astype(F32) * F32(scale) + F32(1.0)
    ch, cw = crop
    sh = (b[:, 2] - b[:, 0]) / F32(ch)
    sw = (b[:, 3] - b[:, 1]) / F32(cw)
    i0, i1 = F32(H + 2 - 1), F32(W + 2 - 1)
    ny = (b[:, 0] + sh / F32(2) - F32(0.5)) / i0
    nx = (b[:, 1] + sw / F32(2) - F32(0.5)) / i1
    nh = sh * F32(ch - 1) / i0
    nw = sw * F32(cw - 1) / i1
    return np.stack([ny, nx, ny + nh, nx + nw], 1).astype(F32)


class _PoolCPU(torch.autograd.Function):
    """ROIPooler (poolers.py:134-180) forward in C, backward as the per-level
    CropAndResizeGradImage + MirrorPadGrad(SYMMETRIC, 1)."""

    @staticmethod
    def forward(ctx, boxes, img, out_size, scales, *levels):
        lv_np = [x.detach().numpy() for x in levels]
        pooled, lv = oracle.roi_pooler(lv_np, boxes, img, out_size, scales, 0, True)
        ctx.meta = (boxes, img, out_size, scales, lv, [x.shape for x in levels])
        return torch.from_numpy(pooled)

    @staticmethod
    def backward(ctx, g):
        boxes, img, out_size, scales, lv, shapes = ctx.meta
        g = g.contiguous().numpy()
        grads = []
        for level, (shp, s) in enumerate(zip(shapes, scales)):
            N, H, W, C = shp
            inds = np.where(lv == level)[0]
            gp = np.zeros((N, H + 2, W + 2, C), F32)
            if inds.size:
                nb = _aligned_boxes(boxes[inds], s, out_size, H, W)
                gp = oracle.crop_and_resize_grad_image(g[inds], nb, img[inds], (N, H + 2, W + 2))
            gp[:, 1] += gp[:, 0]
            gp[:, -2] += gp[:, -1]
            gp[:, :, 1] += gp[:, :, 0]
            gp[:, :, -2] += gp[:, :, -1]
            grads.append(torch.from_numpy(np.ascontiguousarray(gp[:, 1:-1, 1:-1])))
        return (None, None, None, None, *grads)


class CPUTrainStep:
    def __init__(self, model, cfg):
        from detectron2_tensorflow_amd.solver import MomentumSGD, build_learning_rate, param_groups
        self.m = copy.deepcopy(model).cpu().train()
        self.opt = MomentumSGD(param_groups(self.m, cfg), cfg.SOLVER.MOMENTUM,
                               cfg.SOLVER.CLIP_GRADIENTS_BY_NORM)
        self.lr = build_learning_rate(cfg)
        self.iter = 0

    def losses(self, images, image_shapes, gt):
        from detectron2_tensorflow_amd.modeling.roi_heads.fast_rcnn import fast_rcnn_losses
        from detectron2_tensorflow_amd.structures import BoxList, ImageList
        m = self.m
        x = (torch.from_numpy(np.asarray(images, F32)) - m.pixel_mean) / m.pixel_std
        if m.input_format == "BGR":
            x = x.flip(-1)
        H, W = x.shape[1:3]
        d = m.neck.size_divisibility
        x = F.pad(x, (0, 0, 0, (-W) % d, 0, (-H) % d)).contiguous()
        N = x.shape[0]
        feats = _fpn(m.neck, _backbone(m.backbone, x))
        rpn = m.proposal_generator
        head = rpn.rpn_head
        ag = rpn.anchor_generator
        logits, deltas, anchors, props, lg_np = [], [], [], [], []
        for lvl, f in enumerate(rpn.in_features):
            share = _conv(feats[f], head.conv)
            lg = _conv(share, head.objectness_logits)
            dl = _conv(share, head.anchor_deltas)
            h, w = lg.shape[1:3]
            anc = oracle.grid_anchors(h, w, ag.strides[lvl], ag.cell_anchors[lvl].numpy())
            logits.append(lg)
            deltas.append(dl)
            anchors.append(anc)
            p = oracle.apply_deltas(dl.detach().numpy().reshape(-1, 4), np.tile(anc, (N, 1)),
                                    rpn.box2box_transform.weights)
            props.append(p.reshape(N, -1, 4))
            lg_np.append(lg.detach().numpy().reshape(N, -1))
        fl = [feats[f] for f in rpn.in_features]
        rpn._anchors = torch.from_numpy(np.concatenate(anchors))
        rpn._anchor_key = tuple((f.shape[1], f.shape[2]) for f in fl) + (str(fl[0].device),)
        shapes_t = torch.as_tensor(np.asarray(image_shapes), dtype=torch.int32)
        images_l = ImageList(x, shapes_t)
        losses = rpn.losses(images_l, fl, logits, deltas, gt)
        pb, ps, pv = oracle.find_top_rpn_proposals(props, lg_np, np.asarray(image_shapes),
                                                   rpn.nms_thresh, rpn.pre_nms_topk[True],
                                                   rpn.post_nms_topk[True],
                                                   float(rpn.min_box_side_len))
        rh = m.roi_heads
        prop = BoxList(torch.from_numpy(pb))
        prop.add_field("is_valid", torch.from_numpy(pv.astype(bool)))
        s = rh.label_and_sample_proposals(prop, gt)
        S = s["boxes"].shape[1]
        levels = [feats[f] for f in rh.in_features]
        bp = rh.box_pooler
        boxes = s["boxes"].reshape(-1, 4).numpy()
        img = np.repeat(np.arange(N), S).astype(np.int32)
        xb = _PoolCPU.apply(boxes, img, bp.output_size, bp.scales, *levels).reshape(N * S, -1)
        for fc in rh.box_head.fcs:
            xb = torch.relu(xb @ fc.weights + fc.bias)
        cls = xb @ rh.box_predictor.cls_score.weights + rh.box_predictor.cls_score.bias
        dlt = xb @ rh.box_predictor.bbox_pred.weights + rh.box_predictor.bbox_pred.bias
        losses.update(fast_rcnn_losses(cls, dlt, s["boxes"].reshape(-1, 4),
                                       s["gt_classes"].reshape(-1), s["gt_boxes"].reshape(-1, 4),
                                       s["is_valid"].reshape(-1), rh.box2box_transform,
                                       rh.smooth_l1_beta))
        if rh.mask_on:
            Fg = int(rh.batch_size_per_image * rh.positive_sample_fraction)
            mb = s["boxes"][:, :Fg].reshape(-1, 4)
            mcls = s["gt_classes"][:, :Fg].reshape(-1)
            fg = (s["is_valid"][:, :Fg].reshape(-1) & (mcls >= 0) & (mcls < rh.num_classes))
            mp = rh.mask_pooler
            mimg = np.repeat(np.arange(N), Fg).astype(np.int32)
            y = _PoolCPU.apply(mb.numpy(), mimg, mp.output_size, mp.scales, *levels)
            for c in rh.mask_head.convs:
                y = _conv(y, c)
            dc = rh.mask_head.deconv
            y = F.conv_transpose2d(y.permute(0, 3, 1, 2), dc.weights.permute(3, 2, 0, 1), dc.bias,
                                   stride=dc.stride)
            y = torch.relu(y).permute(0, 2, 3, 1)
            y = _conv(y, rh.mask_head.predictor)
            gm = gt["gt_masks"].numpy().astype(F32)
            G = gm.shape[1]
            gidx = (s["gt_index"][:, :Fg] + torch.arange(N)[:, None] * G).reshape(-1).numpy()
            gb = s["gt_boxes"][:, :Fg].reshape(-1, 4).numpy()
            b = mb.numpy()
            gh, gw = gb[:, 2] - gb[:, 0], gb[:, 3] - gb[:, 1]
            with np.errstate(divide="ignore", invalid="ignore"):
                nb = np.stack([(b[:, 0] - gb[:, 0]) / gh, (b[:, 1] - gb[:, 1]) / gw,
                               (b[:, 2] - gb[:, 0]) / gh, (b[:, 3] - gb[:, 1]) / gw], 1)
            fgn = fg.numpy()
            Hm, Wm = y.shape[1:3]
            tgt = np.zeros((len(b), Hm, Wm), F32)
            if fgn.any():
                t = oracle.crop_and_resize_tf(gm.reshape(N * G, *gm.shape[2:])[..., None],
                                              nb[fgn].astype(F32), gidx[fgn].astype(np.int32),
                                              (Hm, Wm))[..., 0]
                tgt[fgn] = np.round(t)
            ch = mcls.clamp(0, y.shape[-1] - 1)
            logit = y[torch.arange(len(b)), :, :, ch]
            bce = F.binary_cross_entropy_with_logits(logit, torch.from_numpy(tgt), reduction="none")
            n = max(int(fg.sum()) * Hm * Wm, 1)
            losses["loss_mask"] = torch.where(fg[:, None, None], bce, torch.zeros_like(bce)).sum() / n
        return losses

    def step(self, images, image_shapes, gt, threads=None):
        if threads:
            torch.set_num_threads(threads)
        self.opt.zero_grad()
        losses = self.losses(images, image_shapes, gt)
        total = sum(losses.values())
        total.backward()
        self.opt.step(self.lr(self.iter))
        self.iter += 1
        return {k: float(v) for k, v in losses.items()}
