"""End-to-end GPU parity: the whole Mask R-CNN R50-FPN inference (HIP hot path)
against the CPU restatement of the reference forward (oracle/cpu_pipeline.py)
with the same weights and image.

Op-level parity is exact (test_gpu_ops.py).  End to end, the fp32 convs on
MFMA vs torch-CPU differ in summation order (~1e-6 relative), which can
reorder near-tied proposals; the bar of the whole-pipeline test is therefore
statistical: RPN proposal sets and final detections agree on >= 95% of
entries, scores within 1e-3 and masks within 1e-3 where the detection
matches.  The stage-wise tests at 1333x800 (Faster R-CNN, C2; Mask R-CNN,
r6) compare every stage against the oracle on the model's own inputs to that
stage, with exact decisions.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model(dev, mask=True):
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    from detectron2_tensorflow_amd.modeling import build_model
    cfg = get_cfg()
    name = ("COCO-InstanceSegmentation/mask_rcnn_R_50_FPN_1x.yaml" if mask
            else "COCO-Detection/faster_rcnn_R_50_FPN_1x.yaml")
    cfg.merge_from_file(os.path.join(ROOT, "configs", name))
    cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT = "raw"
    finalize(cfg, False, 1, {"num_thing_classes": 80, "num_stuff_classes": 53,
                             "stuff_ignore_value": 0})
    torch.manual_seed(0)
    m = build_model(cfg)
    # BASELINE.md score injection: class logits ~ N(0, 3^2)-ish
    with torch.no_grad():
        m.roi_heads.box_predictor.cls_score.weights.normal_(0, 0.05)
    return m.to(dev).eval()


def _match_rate(gb, gc, gv, wb, wc, wv):
    hits, total = 0, int(wv.sum())
    for b, c in zip(wb[wv], wc[wv]):
        d = np.abs(gb[gv] - b).max(axis=1)
        hits += bool(((d < 1e-2) & (gc[gv] == c)).any())
    return hits / max(total, 1)


def test_mask_rcnn_end_to_end_vs_cpu_reference(dev):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from cpu_pipeline import CPUReference
    model = _model(dev)
    rng = np.random.default_rng(7)
    img = rng.uniform(0, 255, size=(2, 256, 320, 3)).astype(np.float32)
    shapes = np.array([[256, 320], [224, 300]], np.int32)
    with torch.no_grad():
        out = model.inference({"image": torch.from_numpy(img).to(dev),
                               "image_shape": torch.from_numpy(shapes).to(dev)})["instances"]
        rpn = model.proposal_generator
    want = CPUReference(model)(img, shapes, threads=8)
    g = {k: v.cpu().numpy() for k, v in out.items()}
    for n in range(2):
        rate = _match_rate(g["boxes"][n], g["classes"][n], g["is_valid"][n], want["boxes"][n],
                           want["classes"][n], want["is_valid"][n])
        assert abs(int(g["is_valid"][n].sum()) - int(want["is_valid"][n].sum())) <= 3
        assert rate >= 0.95, f"image {n}: only {rate:.2%} of detections match"
        both = g["is_valid"][n] & want["is_valid"][n]
        same = both & (g["classes"][n] == want["classes"][n]) & \
            (np.abs(g["boxes"][n] - want["boxes"][n]).max(-1) < 1e-2)
        np.testing.assert_allclose(g["scores"][n][same], want["scores"][n][same], atol=1e-3)
        # a mask is sampled at its detection's box: a box that moved by 1e-2 px
        # moves every ROIAlign sample, so masks are compared where the boxes
        # agree to 1e-3 px (mask-head parity on identical ROIs is the 1e-4
        # test below)
        tight = same & (np.abs(g["boxes"][n] - want["boxes"][n]).max(-1) < 1e-3)
        assert tight.sum() >= 0.8 * same.sum()
        np.testing.assert_allclose(g["masks"][n][tight], want["masks"][n][tight], atol=1e-3)


def test_fpn_and_mask_head_logits_on_identical_inputs(dev):
    """north_star: mask logits within 1e-4 of the reference CPU path on
    identical inputs.  Same res2..res5 features -> FPN p2..p6 (fpn.py:121-183),
    and same pooled ROI features -> mask head logits (mask_head.py:153-170),
    MFMA convs on the GPU vs the CPU restatement (torch-CPU convs, float64 as
    the exact arithmetic); the GPU error is also checked to be no larger than
    the float32 CPU restatement's own error (summation order only)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_pipeline as cp
    import torch.nn.functional as F
    model = _model(dev)
    ref = cp.CPUReference(model)
    g = torch.Generator().manual_seed(3)
    shapes = {"res2": (64, 80, 256), "res3": (32, 40, 512), "res4": (16, 20, 1024),
              "res5": (8, 10, 2048)}
    feats = {k: torch.relu(torch.randn((2,) + v, generator=g)) for k, v in shapes.items()}
    with torch.no_grad():
        got = model.neck({k: v.to(dev) for k, v in feats.items()})
        m64 = ref.m.double()
        want = cp._fpn(m64.neck, {k: v.double() for k, v in feats.items()})
        m32 = cp.CPUReference(model).m
        want32 = cp._fpn(m32.neck, feats)
    for k in want:
        w = want[k]
        err = (got[k].cpu().double() - w).abs().max().item()
        err32 = (want32[k].double() - w).abs().max().item()
        scale = w.abs().max().item()
        assert err <= 1e-4 * max(scale, 1.0), (k, err, scale)
        assert err <= 4 * err32 + 1e-6, (k, err, err32)
    # mask head: 14x14x256 pooled features -> 28x28x80 logits
    x = torch.randn(24, 14, 14, 256, generator=g)
    with torch.no_grad():
        _, logit = model.roi_heads.mask_head(x.to(dev))
        mh = m64.roi_heads.mask_head
        y = x.double()
        for c in mh.convs:
            y = cp._conv(y, c)
        y = F.conv_transpose2d(y.permute(0, 3, 1, 2), mh.deconv.weights.permute(3, 2, 0, 1),
                               mh.deconv.bias, stride=mh.deconv.stride)
        y = cp._conv(torch.relu(y).permute(0, 2, 3, 1), mh.predictor)
    err = (logit.cpu().double() - y).abs().max().item()
    assert logit.shape == (24, 28, 28, 80)
    assert err <= 1e-4 * max(y.abs().max().item(), 1.0), err


def test_faster_rcnn_batch_shapes_and_determinism(dev):
    model = _model(dev, mask=False)
    img = torch.rand(2, 320, 480, 3, device=dev) * 255
    inp = {"image": img, "image_shape": torch.tensor([[320, 480], [300, 470]], device=dev)}
    # every conv of this model runs on the HIP kernels (deterministic:
    # fixed-order split-K, sorted NMS / top-k); the flag only guards a torch
    # fallback conv (MIOpen, whose default solutions include atomic split-K)
    old = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    try:
        with torch.no_grad():
            model.inference(inp)  # first call: MIOpen / hipBLASLt pick their solutions
            a = model.inference(inp)["instances"]
            b = model.inference(inp)["instances"]
    finally:
        torch.backends.cudnn.deterministic = old
    assert a["boxes"].shape == (2, 100, 4) and a["classes"].dtype == torch.int64
    for k in a:
        assert torch.equal(a[k], b[k]), k  # NMS / top-k are deterministic
    v = a["is_valid"]
    assert torch.all(a["boxes"][~v] == 0) and torch.all(a["scores"][~v] == 0)
    # boxes clipped to each image's true shape (fast_rcnn.py:111-116)
    assert torch.all(a["boxes"][0][..., 2] <= 320) and torch.all(a["boxes"][1][..., 3] <= 470)


@pytest.mark.parametrize("fmt", ["conventional", "fixed"])
def test_mask_rcnn_pasted_masks_match_oracle_paste(dev, fmt):
    """SEGMENTATION_OUTPUT.FORMAT conventional / fixed (rcnn.py:124-133 ->
    detector_postprocess): the model's uint8 canvas masks equal the oracle's
    paste (crop_and_resize of the reverse box + tf.greater) of the same run's
    raw 28x28 masks, boxes and validity, bit for bit."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    model = _model(dev)
    rng = np.random.default_rng(11)
    img = rng.uniform(0, 255, size=(2, 256, 320, 3)).astype(np.float32)
    shapes = np.array([[256, 320], [224, 300]], np.int32)
    batch = {"image": torch.from_numpy(img).to(dev), "image_shape": torch.from_numpy(shapes).to(dev)}
    # given detections (inference(detected_instances=...), rcnn.py:118-122):
    # a random-init box regressor sends its own detections to degenerate
    # border boxes, which paste as empty masks
    from detectron2_tensorflow_amd.structures import BoxList
    N, D = 2, 40
    cy, cx = rng.uniform(0, 224, (N, D)), rng.uniform(0, 300, (N, D))
    h, w = rng.uniform(4, 150, (N, D)), rng.uniform(4, 150, (N, D))
    bx = np.stack([cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2], -1).astype(np.float32)
    det = BoxList(torch.from_numpy(bx).to(dev))
    det.add_field("pred_classes", torch.from_numpy(rng.integers(0, 80, (N, D))).to(dev))
    det.add_field("scores", torch.rand(N, D, device=dev))
    det.add_field("is_valid", torch.from_numpy(rng.random((N, D)) < 0.9).to(dev))
    with torch.no_grad():
        raw = model.inference(batch, detected_instances=det)["instances"]
        model.segmentation_output_format = fmt
        pasted = model.inference(batch, detected_instances=det)["instances"]
    model.segmentation_output_format = "raw"
    R = model.segmentation_output_resolution
    H, W = (R, R) if fmt == "fixed" else (256, 320)
    masks = pasted["masks"].cpu().numpy()
    assert masks.shape == (N, D, H, W) and masks.dtype == np.uint8
    for n in range(N):
        yx = None
        if fmt == "fixed":
            yx = (np.array([R, R], np.float64) / shapes[n].astype(np.float64)).astype(np.float32)
            yx = np.repeat(yx[None], D, 0)
        want = oracle.paste_masks(raw["masks"][n].cpu().numpy(), raw["boxes"][n].cpu().numpy(),
                                  (H, W), valid=raw["is_valid"][n].cpu().numpy(), yx_scale=yx)
        np.testing.assert_array_equal(masks[n], want)
    assert masks.sum() > 0


def test_faster_rcnn_c2_1333x800_vs_oracle_on_its_own_heads(dev):
    """Config C2 assembled at its own geometry: Faster R-CNN R50-FPN inference
    (rcnn.py:92-144) on 2 synthetic 1333x800 images (padded to 1344x800),
    BASELINE.md score injection.  (1) two forwards are identical and the
    output has the reference layout (100 slots per image, valid-first,
    scores descending); (2) the RPN proposals equal the oracle's
    find_top_rpn_proposals (rpn_outputs.py:29-132) run on the model's OWN
    RPN-head outputs over all 268,569 anchors per image: scores and valid
    flags bit-exact, boxes within max(1e-4, 2 ulp); (3) the detections equal
    the oracle's fast_rcnn_inference (fast_rcnn.py:28-187) on the model's
    OWN box-head outputs and proposals: valid flags bit-exact, scores within
    2e-6 relative, classes bit-exact and boxes within max(1e-4, 2 ulp) --
    position by position, except among detections whose oracle scores tie
    within that tolerance (compared as sets: their order follows ulp-level
    softmax differences)."""
    import oracle
    from test_gpu_ops import assert_boxes_close
    from detectron2_tensorflow_amd.utils.synthetic import calibrate_rcnn_scores, synthetic_images
    model = _model(dev, mask=False)
    batch = synthetic_images(2, 800, 1333, 1000, dev)
    calibrate_rcnn_scores(model, batch)
    model.eval()
    cap = {}
    pg, rh = model.proposal_generator, model.roi_heads
    hooks = [pg.rpn_head.register_forward_hook(lambda m, i, o: cap.__setitem__("rpn", o)),
             pg.register_forward_hook(lambda m, i, o: cap.__setitem__("props", o[0])),
             rh.box_predictor.register_forward_hook(lambda m, i, o: cap.__setitem__("box", o))]
    try:
        with torch.no_grad():
            a = model.inference(batch)["instances"]
            rpn_out = [[t.detach().contiguous().cpu().numpy() for t in lst] for lst in cap["rpn"][1:]]
            props = cap["props"]
            pboxes = props.boxes.cpu().numpy()
            pscores = props.get_field("objectness_logits").cpu().numpy()
            pvalid = props.get_field("is_valid").cpu().numpy()
            logits, deltas = (t.detach().cpu().numpy() for t in cap["box"])
            b = model.inference(batch)["instances"]
    finally:
        for h in hooks:
            h.remove()
    # (1) determinism and layout
    for k in a:
        assert torch.equal(a[k], b[k]), k
    h = {k: v.cpu().numpy() for k, v in a.items()}
    N, D = h["is_valid"].shape
    assert (N, D) == (2, 100) and h["boxes"].shape == (2, 100, 4)
    for n in range(N):
        v = h["is_valid"][n]
        k = int(v.sum())
        assert k > 0 and v[:k].all() and not v[k:].any()
        assert np.all(np.diff(h["scores"][n][:k]) <= 0)
    # (2) proposals vs the oracle on the model's own RPN-head outputs
    image_hw = batch["image_shape"].cpu().numpy()
    ag = pg.anchor_generator
    lg, dl = rpn_out
    A = lg[0].shape[-1]
    assert sum(x.shape[1] * x.shape[2] * A for x in lg) == 268569
    cells = [np.asarray(c.cpu() if torch.is_tensor(c) else c, np.float32) for c in ag.cell_anchors]
    wprops = []
    for x, d, s, c in zip(lg, dl, ag.strides, cells):
        anc = oracle.grid_anchors(x.shape[1], x.shape[2], s, c)
        wprops.append(oracle.apply_deltas(d.reshape(-1, 4), np.tile(anc, (N, 1)), (1, 1, 1, 1))
                      .reshape(N, -1, 4))
    wb, ws, wv = oracle.find_top_rpn_proposals(
        wprops, [x.reshape(N, -1) for x in lg], image_hw, pg.nms_thresh,
        pg.pre_nms_topk[False], pg.post_nms_topk[False], float(pg.min_box_side_len))
    np.testing.assert_array_equal(pvalid, wv)
    np.testing.assert_array_equal(pscores, ws)
    assert_boxes_close(pboxes, wb)
    # (3) detections vs the oracle's fast_rcnn_inference on the model's own box head
    P = pboxes.shape[1]
    rows = np.nonzero(pvalid.reshape(-1))[0]
    roi_img, roi_slot = rows // P, rows % P
    bw = rh.box2box_transform.weights
    dec = oracle.apply_deltas(deltas[rows], pboxes.reshape(-1, 4)[rows], bw)
    want = oracle.fast_rcnn_inference(dec, oracle.softmax(logits[rows]), roi_img, roi_slot, P,
                                      image_hw, rh.test_score_thresh, rh.test_nms_thresh, D,
                                      rh.test_nms_cls_agnostic)
    for n in range(N):
        wbx, wsc, wc, wvd, wroi = want[n]
        np.testing.assert_array_equal(h["is_valid"][n], wvd)
        np.testing.assert_allclose(h["scores"][n], wsc, rtol=2e-6, atol=1e-7)
        k = int(wvd.sum())
        # detections whose oracle scores lie within the score tolerance of each
        # other form a tie group: their order follows ulp-level softmax
        # differences (ocml vs libm expf), so each group is compared as a set
        # of (class, box); everything else position by position
        g0 = 0
        for i in range(1, k + 1):
            if i < k and wsc[g0] - wsc[i] <= 1e-7 + 2e-6 * abs(wsc[g0]):
                continue
            key = lambda c, b: np.lexsort((b[:, 3], b[:, 2], b[:, 1], b[:, 0], c))  # noqa: E731
            gc, gb = h["classes"][n][g0:i], h["boxes"][n][g0:i]
            oc, ob = wc[g0:i], wbx[g0:i]
            og, oo = key(gc, np.round(gb, 2)), key(oc, np.round(ob, 2))
            np.testing.assert_array_equal(gc[og], oc[oo])
            assert_boxes_close(gb[og], ob[oo])
            g0 = i
        assert_boxes_close(h["boxes"][n][k:], wbx[k:])
        assert k >= 20  # a realistic survivor count (score injection)


def test_mask_rcnn_1333x800_vs_oracle_on_its_own_heads(dev):
    """Mask R-CNN R50-FPN inference at the bench geometry (2 synthetic
    1333x800 images, BASELINE.md score injection), stage by stage against the
    oracle on the model's OWN intermediate outputs -- the exact counterpart of
    the statistical 256x320 end-to-end test above:
    (1) the RPN proposals equal find_top_rpn_proposals on the model's RPN-head
    outputs (scores / valid flags bit-exact); (2) the detections equal
    fast_rcnn_inference on its box-head outputs (classes / valid flags exact);
    (3) the mask pooler's 14x14 features equal the oracle ROIPooler
    (poolers.py:134-180) on the model's own p2..p5 and detection boxes
    (<= 1e-5 relative); (4) the mask logits equal a float64 restatement of
    the mask head on those pooled features (1e-4, the north_star bar); (5) the
    returned 28x28 masks are the sigmoid of the predicted class's logits,
    zeroed on invalid slots (mask_head.py:71-106)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_pipeline as cp
    import oracle
    import torch.nn.functional as F
    from test_gpu_ops import assert_boxes_close
    from detectron2_tensorflow_amd.utils.synthetic import calibrate_rcnn_scores, synthetic_images
    model = _model(dev, mask=True)
    batch = synthetic_images(2, 800, 1333, 1000, dev)
    calibrate_rcnn_scores(model, batch)
    model.eval()
    cap = {}
    pg, rh = model.proposal_generator, model.roi_heads
    hooks = [pg.rpn_head.register_forward_hook(lambda m, i, o: cap.__setitem__("rpn", o)),
             pg.register_forward_hook(lambda m, i, o: cap.__setitem__("props", o[0])),
             rh.box_predictor.register_forward_hook(lambda m, i, o: cap.__setitem__("box", o)),
             model.neck.register_forward_hook(lambda m, i, o: cap.__setitem__("fpn", o)),
             rh.mask_head.register_forward_hook(
                 lambda m, i, o: cap.__setitem__("mask", (i[0].detach().clone(), o[1].detach().clone())))]
    try:
        with torch.no_grad():
            a = model.inference(batch)["instances"]
    finally:
        for hk in hooks:
            hk.remove()
    h = {k: v.cpu().numpy() for k, v in a.items()}
    N, D = h["is_valid"].shape
    image_hw = batch["image_shape"].cpu().numpy()
    # (1) proposals
    props = cap["props"]
    pboxes = props.boxes.cpu().numpy()
    pscores = props.get_field("objectness_logits").cpu().numpy()
    pvalid = props.get_field("is_valid").cpu().numpy()
    lg, dl = [[t.detach().contiguous().cpu().numpy() for t in lst] for lst in cap["rpn"][1:]]
    ag = pg.anchor_generator
    cells = [np.asarray(c.cpu() if torch.is_tensor(c) else c, np.float32) for c in ag.cell_anchors]
    wprops = []
    for x, d, st, c in zip(lg, dl, ag.strides, cells):
        anc = oracle.grid_anchors(x.shape[1], x.shape[2], st, c)
        wprops.append(oracle.apply_deltas(d.reshape(-1, 4), np.tile(anc, (N, 1)), (1, 1, 1, 1))
                      .reshape(N, -1, 4))
    wb, ws, wv = oracle.find_top_rpn_proposals(
        wprops, [x.reshape(N, -1) for x in lg], image_hw, pg.nms_thresh,
        pg.pre_nms_topk[False], pg.post_nms_topk[False], float(pg.min_box_side_len))
    np.testing.assert_array_equal(pvalid, wv)
    np.testing.assert_array_equal(pscores, ws)
    assert_boxes_close(pboxes, wb)
    # (2) detections (tie groups compared as sets, as the C2 test)
    logits, deltas = (t.detach().cpu().numpy() for t in cap["box"])
    P = pboxes.shape[1]
    rows = np.nonzero(pvalid.reshape(-1))[0]
    dec = oracle.apply_deltas(deltas[rows], pboxes.reshape(-1, 4)[rows], rh.box2box_transform.weights)
    want = oracle.fast_rcnn_inference(dec, oracle.softmax(logits[rows]), rows // P, rows % P, P,
                                      image_hw, rh.test_score_thresh, rh.test_nms_thresh, D,
                                      rh.test_nms_cls_agnostic)
    for n in range(N):
        wbx, wsc, wc, wvd, _ = want[n]
        np.testing.assert_array_equal(h["is_valid"][n], wvd)
        np.testing.assert_allclose(h["scores"][n], wsc, rtol=2e-6, atol=1e-7)
        k = int(wvd.sum())
        assert k >= 20
        g0 = 0
        for i in range(1, k + 1):
            if i < k and wsc[g0] - wsc[i] <= 1e-7 + 2e-6 * abs(wsc[g0]):
                continue
            key = lambda c, b: np.lexsort((b[:, 3], b[:, 2], b[:, 1], b[:, 0], c))  # noqa: E731
            gc, gb = h["classes"][n][g0:i], h["boxes"][n][g0:i]
            og, oo = key(gc, np.round(gb, 2)), key(wc[g0:i], np.round(wbx[g0:i], 2))
            np.testing.assert_array_equal(gc[og], wc[g0:i][oo])
            assert_boxes_close(gb[og], wbx[g0:i][oo])
            g0 = i
    # (3) the mask pooler on the model's own maps and detection boxes
    pooled, mlogits = cap["mask"]
    feats = [cap["fpn"][f].detach().cpu().numpy() for f in rh.in_features]
    boxes = h["boxes"].reshape(-1, 4)
    img = np.repeat(np.arange(N, dtype=np.int32), D)
    scales = [float(v) for v in rh.mask_pooler.scales]
    R = rh.mask_pooler.output_size
    want_x, _ = oracle.roi_pooler(feats, boxes, img, R, scales, rh.mask_pooler.sampling_ratio)
    got_x = pooled.cpu().numpy().reshape(want_x.shape)
    scale = max(1.0, float(np.abs(want_x).max()))
    assert np.abs(got_x - want_x).max() <= 1e-5 * scale
    # (4) mask logits vs a float64 restatement of the head on those features
    ref = cp.CPUReference(model)
    mh = ref.m.double().roi_heads.mask_head
    with torch.no_grad():
        y = pooled.cpu().double()
        for c in mh.convs:
            y = cp._conv(y, c)
        y = F.conv_transpose2d(y.permute(0, 3, 1, 2), mh.deconv.weights.permute(3, 2, 0, 1),
                               mh.deconv.bias, stride=mh.deconv.stride)
        y = cp._conv(torch.relu(y).permute(0, 2, 3, 1), mh.predictor)
    err = (mlogits.cpu().double() - y).abs().max().item()
    assert err <= 1e-4 * max(y.abs().max().item(), 1.0), err
    # (5) the masks: sigmoid of the predicted class's logits, zero where invalid
    ml = mlogits.cpu()
    cls = torch.from_numpy(h["classes"].reshape(-1)).long().clamp(min=0)
    want_m = torch.sigmoid(ml[torch.arange(ml.shape[0]), :, :, cls])
    want_m = want_m * torch.from_numpy(h["is_valid"].reshape(-1))[:, None, None].float()
    got_m = a["masks"].cpu().reshape(want_m.shape)
    assert torch.allclose(got_m, want_m, rtol=0, atol=2e-7), float((got_m - want_m).abs().max())
