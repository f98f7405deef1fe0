"""detectron2 -> reference (TF) variable names and layouts.

Restates lib/convert_models/convert_d2.py:4-187 on a dict of numpy arrays:
  * conv weights OIHW -> HWIO (transpose 2, 3, 1, 0); ConvTranspose IOHW ->
    [kh, kw, out, in] by the same transpose (TF conv2d_transpose layout);
  * norm.weight / bias -> norm/gamma / beta, running_var / mean ->
    norm/moving_variance / moving_mean (num_batches_tracked dropped);
  * FC weights transposed to [in, out]; fc1's rows reordered from detectron2's
    (C, h, w) flattening to the reference's NHWC (h, w, C) flattening;
  * box-regression outputs (RPN anchor_deltas, box_predictor bbox_pred,
    RetinaNet bbox_pred) permuted from (x1, y1, x2, y2) to (y1, x1, y2, x2)
    per anchor / class (get_box_indices);
  * every source key must be consumed (cell_anchors buffers excepted).
"""
import numpy as np


def _box_indices(n):
    """convert_d2.py:69-76: per group of 4, detectron2 (dx, dy, dw, dh) order
    -> (dy, dx, dh, dw)."""
    x0 = np.arange(n) * 4
    return np.stack([x0 + 1, x0, x0 + 3, x0 + 2], axis=-1).reshape(n * 4)


def convert_weights(d, cfg):
    """d: {detectron2 name: np.ndarray} (consumed); returns {reference name: array}."""
    d = dict(d)
    has_fpn = cfg.MODEL.NECK.NAME == "FPN"
    use_res5_in_stage2 = cfg.MODEL.ROI_HEADS.NAME == "Res5ROIHeads"
    is_retina = cfg.MODEL.NECK.TOP_BLOCK_TYPE == "P6P7"
    ret = {}

    def conv(src, dst):
        ret[dst + "/weights"] = np.ascontiguousarray(d.pop(src + ".weight").transpose(2, 3, 1, 0))
        if src + ".norm.weight" in d:
            ret[dst + "/norm/gamma"] = d.pop(src + ".norm.weight")
            ret[dst + "/norm/beta"] = d.pop(src + ".norm.bias")
        if src + ".norm.running_var" in d:
            ret[dst + "/norm/moving_variance"] = d.pop(src + ".norm.running_var")
            ret[dst + "/norm/moving_mean"] = d.pop(src + ".norm.running_mean")
            d.pop(src + ".norm.num_batches_tracked", None)
        if src + "_offset.weight" in d:
            ret[dst + "/offset_weights"] = d.pop(src + "_offset.weight").transpose(2, 3, 1, 0)
            ret[dst + "/offset_bias"] = d.pop(src + "_offset.bias")
        if src + ".bias" in d:
            ret[dst + "/bias"] = d.pop(src + ".bias")

    def fc(src, dst):
        ret[dst + "/weights"] = np.ascontiguousarray(d.pop(src + ".weight").transpose())
        ret[dst + "/bias"] = d.pop(src + ".bias")

    src_prefix = "backbone.bottom_up." if has_fpn else "backbone."
    dst_prefix = "backbone/"
    conv(src_prefix + "stem.conv1", dst_prefix + "stem/conv1")
    blocks = {50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}[cfg.MODEL.RESNETS.DEPTH]
    for g in range(4):
        if use_res5_in_stage2 and g == 3 and not is_retina:
            src_prefix, dst_prefix = "roi_heads.", "roi_heads/"
        for b in range(blocks[g]):
            for c in ("conv1", "conv2", "conv3") + (("shortcut",) if b == 0 else ()):
                conv(f"{src_prefix}res{g + 2}.{b}.{c}", f"{dst_prefix}res{g + 2}/block_{b + 1}/{c}")
    if is_retina:
        for lvl in (6, 7):
            conv(f"backbone.top_block.p{lvl}", f"neck/top_block/p{lvl}")
        for lvl in (3, 4, 5):
            conv(f"backbone.fpn_lateral{lvl}", f"neck/fpn_lateral{lvl}")
            conv(f"backbone.fpn_output{lvl}", f"neck/fpn_output{lvl}")
    elif has_fpn:
        for lvl in (2, 3, 4, 5):
            conv(f"backbone.fpn_lateral{lvl}", f"neck/fpn_lateral{lvl}")
            conv(f"backbone.fpn_output{lvl}", f"neck/fpn_output{lvl}")

    if is_retina:
        for i in range(cfg.MODEL.RETINANET.NUM_CONVS):
            conv(f"head.cls_subnet.{2 * i}", f"head/cls_subnet{2 * i}")
            conv(f"head.bbox_subnet.{2 * i}", f"head/bbox_subnet{2 * i}")
        conv("head.cls_score", "head/cls_score")
        conv("head.bbox_pred", "head/bbox_pred")
        idx = _box_indices(ret["head/bbox_pred/bias"].shape[0] // 4)
        ret["head/bbox_pred/bias"] = ret["head/bbox_pred/bias"][idx]
        ret["head/bbox_pred/weights"] = np.ascontiguousarray(ret["head/bbox_pred/weights"][..., idx])
    elif cfg.MODEL.META_ARCHITECTURE != "SemanticSegmentor":
        src, dst = "proposal_generator.rpn_head", "proposal_generator/rpn_head"
        conv(src + ".conv", dst + "/share")
        conv(src + ".objectness_logits", dst + "/objectness_logits")
        conv(src + ".anchor_deltas", dst + "/anchor_deltas")
        idx = _box_indices(ret[dst + "/objectness_logits/bias"].shape[0])
        ret[dst + "/anchor_deltas/bias"] = ret[dst + "/anchor_deltas/bias"][idx]
        ret[dst + "/anchor_deltas/weights"] = np.ascontiguousarray(
            ret[dst + "/anchor_deltas/weights"][..., idx])

        def box_predictor(src, dst):
            n = 1 if cfg.MODEL.ROI_BOX_HEAD.CLS_AGNOSTIC_BBOX_REG else cfg.MODEL.ROI_HEADS.NUM_CLASSES
            idx = _box_indices(n)
            ret[dst + "/box_deltas/bias"] = d.pop(src + ".bbox_pred.bias")[idx]
            ret[dst + "/box_deltas/weights"] = np.ascontiguousarray(
                d.pop(src + ".bbox_pred.weight").transpose()[..., idx])
            fc(src + ".cls_score", dst + "/class_logits")

        h = cfg.MODEL.ROI_BOX_HEAD
        res = h.POOLER_RESOLUTION
        fc_in = cfg.MODEL.NECK.OUT_CHANNELS if has_fpn else cfg.MODEL.RESNETS.RES2_OUT_CHANNELS * 8
        if h.NUM_CONV > 0:
            fc_in = h.CONV_DIM

        def fc1_nhwc(name):  # (C, h, w) rows -> (h, w, C) rows
            w = ret[name].reshape(fc_in, res, res, -1).transpose(1, 2, 0, 3)
            ret[name] = np.ascontiguousarray(w.reshape(res * res * fc_in, -1))

        cascade = cfg.MODEL.ROI_HEADS.NAME in ("CascadeROIHeads", "CascadeLCCHeads")
        if cascade:
            assert h.CLS_AGNOSTIC_BBOX_REG
            for k in range(3):
                for i in range(h.NUM_CONV):
                    conv(f"roi_heads.box_head.{k}.conv{i + 1}", f"roi_heads/box_head_stage{k + 1}/conv{i + 1}")
                for i in range(h.NUM_FC):
                    fc(f"roi_heads.box_head.{k}.fc{i + 1}", f"roi_heads/box_head_stage{k + 1}/fc{i + 1}")
                    if i == 0:
                        fc1_nhwc(f"roi_heads/box_head_stage{k + 1}/fc1/weights")
                box_predictor(f"roi_heads.box_predictor.{k}", f"roi_heads/box_predictor_stage{k + 1}")
        else:
            for i in range(h.NUM_CONV):
                conv(f"roi_heads.box_head.conv{i + 1}", f"roi_heads/box_head/conv{i + 1}")
            for i in range(h.NUM_FC):
                fc(f"roi_heads.box_head.fc{i + 1}", f"roi_heads/box_head/fc{i + 1}")
                if i == 0:
                    fc1_nhwc("roi_heads/box_head/fc1/weights")
            box_predictor("roi_heads.box_predictor",
                          "roi_heads/fastrcnn" if use_res5_in_stage2 else "roi_heads/box_predictor")
        if cfg.MODEL.MASK_ON:
            for i in range(cfg.MODEL.ROI_MASK_HEAD.NUM_CONV):
                conv(f"roi_heads.mask_head.mask_fcn{i + 1}", f"roi_heads/mask_head/mask_fcn{i + 1}")
            conv("roi_heads.mask_head.deconv", "roi_heads/mask_head/deconv")
            conv("roi_heads.mask_head.predictor", "roi_heads/mask_head/predictor")

    if cfg.MODEL.META_ARCHITECTURE in ("PanopticFPN", "SemanticSegmentor"):
        for i, feat in enumerate(cfg.MODEL.SEM_SEG_HEAD.IN_FEATURES):
            n = max(1, int(i + 2 - np.log2(cfg.MODEL.SEM_SEG_HEAD.COMMON_STRIDE)))
            for k in range(n):
                conv(f"sem_seg_head.{feat}.{2 * k}", f"sem_seg_head/{feat}_{2 * k}")
        conv("sem_seg_head.predictor", "sem_seg_head/predictor")

    for k in [k for k in d if "cell_anchors" in k]:
        d.pop(k)
    if d:
        raise ValueError(f"unconverted detectron2 keys: {sorted(d)[:10]} ...")
    return ret
