"""ORACLE — test infrastructure only.  End-to-end CPU restatement of the
reference's Mask R-CNN / Faster R-CNN R50-FPN inference
(lib/modeling/meta_arch/rcnn.py:92-157) with the weights of a built model:

  preprocess (rcnn.py:146-157) -> ResNet (the model's own backbone module on
  CPU torch convs: the backbone is a caller of the hot path) -> FPN with
  torch-CPU convs + nearest upsample (fpn.py:121-159) -> RPN head convs ->
  ALL anchors materialised and decoded (anchor_generator.py:92-109,
  rpn_outputs.py:403-426) -> find_top_rpn_proposals (rpn_outputs.py:29-132)
  -> per-level ROIAlign with a materialised SYMMETRIC pad (poolers.py:134-180)
  -> box head GEMMs -> softmax/decode/fast_rcnn_inference (fast_rcnn.py:28-187)
  -> mask pooler + mask head convs + mask_rcnn_inference (mask_head.py:71-103).

It is what bench.py times as ``cpu_baseline`` (kind "port": a TF-1.15
semantics restatement, not TensorFlow) and what the end-to-end parity test
compares the GPU model against.  Never imported by the product path.
"""
import copy
import os

import numpy as np
import torch
import torch.nn.functional as F

import oracle
import solo

F32 = np.float32


def _conv(x_nhwc, layer, relu=None, stride=None):
    """Reference Conv2D.call on CPU (convolutional.py:198-263): fix_padding +
    VALID conv + bias, then the normalizer (FrozenBN: (x - mean) * gamma /
    sqrt(var + eps) + beta), then the activation."""
    k = layer.kernel_size
    s = stride or layer.stride
    x = x_nhwc
    if layer.padding == "SAME" and k != 1:
        pt = k - 1
        x = F.pad(x, (0, 0, pt // 2, pt - pt // 2, pt // 2, pt - pt // 2))
    y = F.conv2d(x.permute(0, 3, 1, 2), layer.weights.permute(3, 2, 0, 1), layer.bias, stride=s)
    y = y.permute(0, 2, 3, 1)
    bn = layer.normalizer_fn
    if bn is not None:
        y = (y - bn.moving_mean) * (bn.gamma / torch.sqrt(bn.moving_variance + bn.epsilon)) + bn.beta
    act = layer.act_fn if relu is None else (torch.relu if relu else None)
    return act(y) if act is not None else y


def _backbone(bb, x):
    """ResNet.call (resnet.py:238-253): stem conv + zero pad + 3x3/2 VALID max
    pool, then bottlenecks relu(conv3(conv2(conv1(x))) + shortcut(x))."""
    outs = {}
    y = _conv(x, bb.stem.conv1)
    y = F.max_pool2d(F.pad(y.permute(0, 3, 1, 2), (1, 1, 1, 1)), 3, 2).permute(0, 2, 3, 1)
    for name, stage in zip(bb.stage_names, bb.stages):
        for blk in stage.blocks:
            sc = _conv(y, blk.shortcut) if blk.shortcut is not None else y
            y = torch.relu(_conv(_conv(_conv(y, blk.conv1), blk.conv2), blk.conv3) + sc)
        if name in bb._out_features:
            outs[name] = y
    return outs


def _fpn(neck, x_feats):
    """FPN.call (fpn.py:121-159) + LastLevelMaxPool (fpn.py:171-183) or
    LastLevelP6P7 (fpn.py:186-217: p6 = ReLU(conv3x3/2(res5)) — the post-ReLU
    p6 is what the head sees — and p7 = conv3x3/2(p6), no activation)."""
    x = [x_feats[f] for f in neck.in_features[::-1]]
    prev = _conv(x[0], neck.lateral_convs[0])
    results = [_conv(prev, neck.output_convs[0])]
    for f, lat, out in zip(x[1:], neck.lateral_convs[1:], neck.output_convs[1:]):
        top = prev.repeat_interleave(2, 1).repeat_interleave(2, 2)
        prev = _conv(f, lat) + top
        results.insert(0, _conv(prev, out))
    tb = neck.top_block_type
    if tb == "MAXPOOL":
        results.append(results[-1][:, ::2, ::2, :])  # max_pool k1 s2 VALID
    elif tb == "P6P7":
        p6 = _conv(x_feats["res5"], neck.top_block.p6)
        results.extend([p6, _conv(p6, neck.top_block.p7)])
    return dict(zip(neck._out_features, results))


class CPUReference:
    def __init__(self, model):
        self.m = copy.deepcopy(model).cpu().eval()
        for p in self.m.parameters():
            p.requires_grad_(False)

    def fpn(self, feats):
        return _fpn(self.m.neck, feats)

    @torch.no_grad()
    def __call__(self, images, image_shapes, threads=None, paste_to=None):
        if threads:
            torch.set_num_threads(threads)
        m = self.m
        x = (torch.from_numpy(np.asarray(images, F32)) - m.pixel_mean) / m.pixel_std
        if m.input_format == "BGR":
            x = x.flip(-1)
        H, W = x.shape[1:3]
        d = m.neck.size_divisibility
        x = F.pad(x, (0, 0, 0, (-W) % d, 0, (-H) % d))
        feats = self.fpn(_backbone(m.backbone, x.contiguous()))
        rpn = m.proposal_generator
        head = rpn.rpn_head
        N = x.shape[0]
        props, logits = [], []
        ag = rpn.anchor_generator
        for lvl, f in enumerate(rpn.in_features):
            share = _conv(feats[f], head.conv)
            lg = _conv(share, head.objectness_logits).numpy()
            dl = _conv(share, head.anchor_deltas).numpy()
            h, w = lg.shape[1:3]
            anc = oracle.grid_anchors(h, w, ag.strides[lvl], ag.cell_anchors[lvl].numpy())
            p = oracle.apply_deltas(dl.reshape(-1, 4), np.tile(anc, (N, 1)),
                                    rpn.box2box_transform.weights)
            props.append(p.reshape(N, -1, 4))
            logits.append(lg.reshape(N, -1))
        shapes = np.asarray(image_shapes)
        pb, ps, pv = oracle.find_top_rpn_proposals(props, logits, shapes, rpn.nms_thresh,
                                                   rpn.pre_nms_topk[False],
                                                   rpn.post_nms_topk[False],
                                                   float(rpn.min_box_side_len))
        rh = m.roi_heads
        P = pb.shape[1]
        roi_img, roi_slot = np.nonzero(pv)
        boxes = pb[roi_img, roi_slot]
        levels = [feats[f].numpy() for f in rh.in_features]
        bp = rh.box_pooler
        pooled, _ = oracle.roi_pooler(levels, boxes, roi_img, bp.output_size, bp.scales,
                                      bp.sampling_ratio, bp.aligned)
        xb = torch.from_numpy(pooled).reshape(len(boxes), -1)
        for fc in rh.box_head.fcs:
            xb = torch.relu(xb @ fc.weights + fc.bias)
        cls = (xb @ rh.box_predictor.cls_score.weights + rh.box_predictor.cls_score.bias).numpy()
        dlt = (xb @ rh.box_predictor.bbox_pred.weights + rh.box_predictor.bbox_pred.bias).numpy()
        probs = oracle.softmax(cls)
        dec = oracle.apply_deltas(dlt, boxes, rh.box2box_transform.weights)
        res = oracle.fast_rcnn_inference(dec, probs, roi_img, roi_slot, P, shapes,
                                         rh.test_score_thresh, rh.test_nms_thresh,
                                         rh.test_detections_per_img)
        out = {"boxes": np.stack([r[0] for r in res]), "scores": np.stack([r[1] for r in res]),
               "classes": np.stack([r[2] for r in res]), "is_valid": np.stack([r[3] for r in res]),
               "rpn": (pb, ps, pv)}
        if rh.mask_on:
            D = out["boxes"].shape[1]
            di, ds = np.nonzero(out["is_valid"])
            mp = rh.mask_pooler
            pooled, _ = oracle.roi_pooler(levels, out["boxes"][di, ds], di, mp.output_size,
                                          mp.scales, mp.sampling_ratio, mp.aligned)
            y = torch.from_numpy(pooled)
            for c in rh.mask_head.convs:
                y = _conv(y, c)
            dc = rh.mask_head.deconv
            y = F.conv_transpose2d(y.permute(0, 3, 1, 2), dc.weights.permute(3, 2, 0, 1), dc.bias,
                                   stride=dc.stride)
            y = torch.relu(y).permute(0, 2, 3, 1)
            y = _conv(y, rh.mask_head.predictor).numpy()
            cls_k = out["classes"][di, ds]
            logit = y[np.arange(len(di)), :, :, cls_k] if y.shape[-1] > 1 else y[..., 0]
            masks = np.zeros((N, D) + logit.shape[1:], F32)
            masks[di, ds] = oracle.sigmoid(logit)
            out["masks"] = masks
            if paste_to is not None:  # detector_postprocess "conventional"
                out["masks"] = np.stack([
                    oracle.paste_masks(masks[n], out["boxes"][n], paste_to, valid=out["is_valid"][n])
                    for n in range(N)])
        return out


class CPURetinaNet:
    """SingleStageDetector + RetinaNetHead inference on CPU
    (single_stage_detector.py:33-83, retinanet.py:110-145, :285-387,
    :418-450): preprocess -> ResNet -> FPN with the P6P7 top block -> box tower
    (NUM_CONVS x conv3x3+ReLU per branch, cls_score / bbox_pred conv3x3) ->
    ALL anchors materialised per level (anchor_generator.py:92-109) ->
    oracle.retinanet_inference (per level sigmoid + top_k(1000) + 0.05
    threshold + decode with MODEL.RPN.BBOX_REG_WEIGHTS, class-offset NMS,
    pad to DETECTIONS_PER_IMAGE)."""

    def __init__(self, model):
        self.m = copy.deepcopy(model).cpu().eval()
        for p in self.m.parameters():
            p.requires_grad_(False)

    def features(self, images):
        m = self.m
        x = (torch.from_numpy(np.asarray(images, F32)) - m.pixel_mean) / m.pixel_std
        if m.input_format == "BGR":
            x = x.flip(-1)
        H, W = x.shape[1:3]
        d = m.neck.size_divisibility
        x = F.pad(x, (0, 0, 0, (-W) % d, 0, (-H) % d))
        return _fpn(m.neck, _backbone(m.backbone, x.contiguous()))

    def head(self, feats):
        """RetinaNetBoxTower.call (retinanet.py:431-450): [N,H,W,A*K], [N,H,W,A*4]."""
        det = self.m.detector
        tower = det.head
        cls, box = [], []
        for f in det.in_features:
            y = feats[f]
            for c in tower.cls_layers:
                y = _conv(y, c)
            cls.append(_conv(y, tower.cls_score))
            y = feats[f]
            for c in tower.box_layers:
                y = _conv(y, c)
            box.append(_conv(y, tower.bbox_pred))
        return cls, box

    def postprocess(self, cls, box):
        """RetinaNetHead.inference on given head outputs (numpy or torch)."""
        det = self.m.detector
        ag = det.anchor_generator
        K = det.num_classes
        cls = [np.asarray(c, F32) for c in cls]
        box = [np.asarray(b, F32) for b in box]
        N = cls[0].shape[0]
        anchors = [oracle.grid_anchors(c.shape[1], c.shape[2], ag.strides[i],
                                       ag.cell_anchors[i].numpy())
                   for i, c in enumerate(cls)]
        res = oracle.retinanet_inference([c.reshape(N, -1, K) for c in cls],
                                         [b.reshape(N, -1, 4) for b in box], anchors, K,
                                         det.topk_candidates, det.score_threshold,
                                         det.nms_threshold, det.max_detections_per_image,
                                         det.box2box_transform.weights,
                                         det.box2box_transform.scale_clamp)
        return {"boxes": np.stack([r[0] for r in res]), "scores": np.stack([r[1] for r in res]),
                "classes": np.stack([r[2] for r in res]),
                "is_valid": np.stack([r[3] for r in res])}

    @torch.no_grad()
    def __call__(self, images, image_shapes=None, threads=None):
        if threads:
            torch.set_num_threads(threads)
        cls, box = self.head(self.features(images))
        out = self.postprocess([c.numpy() for c in cls], [b.numpy() for b in box])
        out["head"] = (cls, box)
        return out


def _group_norm(x, gn):
    """GroupNorm.call (normalization.py:235-260): tf.nn.moments over (H, W,
    group channels) — mean, then mean of squared differences — and
    tf.nn.batch_normalization: inv = rsqrt(var + eps) * gamma,
    x * inv + (beta - mean * inv)."""
    N, H, W, C = x.shape
    G = gn.num_groups
    xr = x.reshape(N, H, W, G, C // G)
    mean = xr.mean(dim=(1, 2, 4), keepdim=True)
    var = ((xr - mean) ** 2).mean(dim=(1, 2, 4), keepdim=True)
    inv = torch.rsqrt(var + gn.epsilon) * gn.gamma.reshape(1, 1, 1, G, C // G)
    y = xr * inv + (gn.beta.reshape(1, 1, 1, G, C // G) - mean * inv)
    return y.reshape(N, H, W, C)


def _conv_gn(x, layer):
    """Conv2D.call with a GroupNorm normalizer (conv -> GN -> activation)."""
    from detectron2_tensorflow_amd.layers import GroupNorm
    if not isinstance(layer.normalizer_fn, GroupNorm):
        return _conv(x, layer)
    k = layer.kernel_size
    if layer.padding == "SAME" and k != 1:
        pt = k - 1
        x = F.pad(x, (0, 0, pt // 2, pt - pt // 2, pt // 2, pt - pt // 2))
    y = F.conv2d(x.permute(0, 3, 1, 2), layer.weights.permute(3, 2, 0, 1), layer.bias,
                 stride=layer.stride).permute(0, 2, 3, 1)
    y = _group_norm(y, layer.normalizer_fn)
    return layer.act_fn(y) if layer.act_fn is not None else y


def _resize(x, hw):
    return torch.from_numpy(solo.resize_bilinear_tf(x.numpy(), int(hw[0]), int(hw[1])))


class CPUSOLOv2:
    """SingleStageDetector + SOLOv2Head inference on CPU
    (single_stage_detector.py:33-83, solo_v2.py:67-721): preprocess -> ResNet
    -> FPN (p2..p6, LastLevelMaxPool) -> MaskKernelBranch (split_features with
    TF bilinear resizes :221-239, coordinate channels + resize to the S x S
    grid :255-266, conv/GN/ReLU towers, solo_cate / solo_kernel, sigmoid +
    point NMS :267-271) -> MaskFeatureBranch (:705-721) -> inference per image
    (:476-565, oracle/solo.py) -> masks to the padded image and boxes
    (:598-623)."""

    def __init__(self, model):
        self.m = copy.deepcopy(model).cpu().eval()
        for p in self.m.parameters():
            p.requires_grad_(False)

    features = CPURetinaNet.features

    def kernel_branch(self, feats):
        """(category logits [N,S,S,K], kernels [N,S,S,D]) per level."""
        b = self.m.detector.mask_kernel_branch
        f = [feats[k] for k in b.in_features]
        f = [_resize(f[0], f[1].shape[1:3]), f[1], f[2], f[3], _resize(f[4], f[3].shape[1:3])]
        cls, ker = [], []
        for i, x in enumerate(f):
            N, H, W, _ = x.shape
            S = b.num_grids[i]
            feat = torch.cat([x, torch.from_numpy(solo.coord_channels(N, H, W))], dim=3)
            feat = _resize(feat, (S, S))
            y = feat[..., :-2]
            for c in b.cls_layers:
                y = _conv_gn(y, c)
            cls.append(_conv(y, b.solo_cate))
            y = feat
            for c in b.kernel_layers:
                y = _conv_gn(y, c)
            ker.append(_conv(y, b.solo_kernel))
        return cls, ker

    def feature_branch(self, feats):
        fb = self.m.detector.mask_feature_branch
        res = None
        for i, f in enumerate(fb.in_features):
            x = feats[f]
            if i > 0 and f == fb.in_features[-1]:
                N, H, W, _ = x.shape
                x = torch.cat([x, torch.from_numpy(solo.coord_channels(N, H, W))], dim=3)
            for layer in fb.scale_heads[i]._layers:
                if hasattr(layer, "kernel_size"):
                    x = _conv_gn(x, layer)
                else:  # Upsample: nearest x2 (wrappers.py:104-116 ignores method)
                    x = x.repeat_interleave(2, 1).repeat_interleave(2, 2)
            res = x if res is None else res + x
        return _conv_gn(res, fb.predictor)

    def postprocess(self, cls, ker, mask_feats, out_hw, cell_logits=None, probs=None):
        """MaskKernelBranch.inference (:476-627) on given head outputs.
        cell_logits(n, cells) -> [len(cells), P] overrides the dynamic conv and
        probs [N, T, K] the sigmoid + point NMS (the tail-parity test feeds the
        GPU's own values: expf differs from numpy's exp by <= 1 ulp)."""
        b = self.m.detector.mask_kernel_branch
        cls = [np.asarray(c, F32) for c in cls]
        ker = [np.asarray(k, F32) for k in ker]
        mf = np.asarray(mask_feats, F32)
        N, Hm, Wm, D = mf.shape
        K = cls[0].shape[-1]
        if probs is None:
            probs = np.concatenate([solo.point_nms(oracle.sigmoid(c)).reshape(N, -1, K)
                                    for c in cls], axis=1)
        probs = np.asarray(probs, F32)
        kern = np.concatenate([k.reshape(N, -1, D) for k in ker], axis=1)
        strides = solo.cell_strides(b.num_grids, b.strides)
        OH, OW = int(out_hw[0]), int(out_hw[1])
        out = {"masks": [], "boxes": [], "classes": [], "scores": [], "is_valid": [], "info": []}
        for n in range(N):
            if cell_logits is None:
                fn = (lambda cells, n=n: (kern[n][cells].astype(np.float64)
                                          @ mf[n].reshape(-1, D).astype(np.float64).T).astype(F32))
            else:
                fn = (lambda cells, n=n: cell_logits(n, cells))
            m, c, s, v, info = solo.inference_single_image(
                probs[n], fn, strides, b.score_threshold, b.mask_threshold,
                b.update_score_threshold, b.pre_nms_topk, b.max_detections_per_image,
                b.nms_kernel, b.nms_sigma)
            im, bx = solo.masks_to_image(m, Hm, Wm, OH, OW, b.mask_threshold)
            for key, val in (("masks", im), ("boxes", bx), ("classes", c), ("scores", s),
                             ("is_valid", v), ("info", info)):
                out[key].append(val)
        for key in ("masks", "boxes", "classes", "scores", "is_valid"):
            out[key] = np.stack(out[key])
        out["probs"] = probs
        return out

    @torch.no_grad()
    def __call__(self, images, image_shapes=None, threads=None):
        if threads:
            torch.set_num_threads(threads)
        feats = self.features(images)
        cls, ker = self.kernel_branch(feats)
        mf = self.feature_branch(feats)
        H, W = feats["p2"].shape[1] * 4, feats["p2"].shape[2] * 4
        out = self.postprocess([c.numpy() for c in cls], [k.numpy() for k in ker], mf.numpy(),
                               (H, W))
        out["head"] = (cls, ker, mf)
        return out


def cpu_cores():
    """CPUs this process may actually use: the affinity mask, capped by a
    cgroup-v2 CPU quota and by OMP_NUM_THREADS when set (on the GPU box the
    affinity mask shows the whole machine while the job gets a share of it)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return n
