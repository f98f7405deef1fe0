"""RetinaNet model path (BASELINE configs C1 and C4): SingleStageDetector +
RetinaNetHead (lib/modeling/meta_arch/single_stage_detector.py:33-83,
lib/modeling/single_stage_heads/retinanet.py:110-145, :285-387, :418-450).

C1 — R50-FPN forward of one synthetic 640x640 image on the CPU restatement
(oracle/cpu_pipeline.py: CPURetinaNet; the reference config is CPU plumbing).
C4 — the GPU path: R50 at 640x640 against the CPU restatement (head outputs,
post-processing bit-exact on identical head outputs, detections end to end),
and R101-FPN at 1333x800 (201,600 anchors x 80 classes = 16.1 M sigmoid
scores per image) against the oracle's post-processing on the GPU's own head
outputs, plus determinism and the padded output layout.

Random-init weights give logits of std ~20 (every sigmoid saturates at 1.0):
the cls_score / bbox_pred weights are rescaled once so logits ~ N(-3, 1) and
deltas ~ N(0, 0.1^2) (BASELINE.md score injection), on both sides.
"""
import os

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
F32 = np.float32
CM = {"num_thing_classes": 80, "num_stuff_classes": 53, "stuff_ignore_value": 0}


def _cfg(depth=50):
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    cfg = get_cfg()
    name = "retinanet_R_50_FPN_1x.yaml" if depth == 50 else "retinanet_R_101_FPN_3x.yaml"
    cfg.merge_from_file(os.path.join(ROOT, "configs", "COCO-Detection", name))
    finalize(cfg, False, 1, CM)
    return cfg


def _model(depth=50):
    from detectron2_tensorflow_amd.modeling import build_model
    torch.manual_seed(0)
    return build_model(_cfg(depth)).eval()


def _check_layout(boxes, scores, classes, valid, num_classes=80):
    """pad_or_clip_boxlist layout (retinanet.py:365-367): the kept detections
    first, in NMS selection order (scores non-increasing), zeros after."""
    for n in range(valid.shape[0]):
        v = valid[n]
        m = int(v.sum())
        assert v[:m].all() and not v[m:].any()
        assert (boxes[n][m:] == 0).all() and (scores[n][m:] == 0).all()
        assert (np.diff(scores[n][:m]) <= 0).all()
        assert ((classes[n][:m] >= 0) & (classes[n][:m] < num_classes)).all()
        assert np.isfinite(boxes[n][:m]).all()


def _same_class_overlap_ok(boxes, classes, valid, thr=0.5):
    """No two kept detections of one class overlap by IoU > thr (the class-offset
    NMS of retinanet.py:349-355)."""
    import oracle
    for n in range(valid.shape[0]):
        m = int(valid[n].sum())
        b, c = boxes[n][:m], classes[n][:m]
        for k in np.unique(c):
            bb = b[c == k]
            if len(bb) < 2:
                continue
            keep = oracle.nms(bb, np.linspace(1, 0, len(bb), dtype=F32), len(bb), thr)
            assert len(keep) == len(bb)


# ---------------------------------------------------------------- C1 (CPU)
def test_c1_retinanet_r50_640_cpu_plumbing():
    """C1: one synthetic 640x640 image through the CPU restatement of the
    RetinaNet R50-FPN forward: 76,725 anchors, a full
    [1, 100] padded result with the reference layout."""
    import cpu_pipeline as cp
    from detectron2_tensorflow_amd.utils.synthetic import calibrate_retinanet_head
    model = _model(50)
    ref = cp.CPURetinaNet(model)
    img = np.random.default_rng(0).uniform(0, 255, (1, 640, 640, 3)).astype(F32)
    with torch.no_grad():
        cls, box = ref.head(ref.features(img))
        calibrate_retinanet_head(ref.m.detector.head, cls, box)
        cls, box = ref.head(ref.features(img))
    A, K = 9, 80
    assert sum(c.shape[1] * c.shape[2] * A for c in cls) == 76725
    assert [c.shape[-1] for c in cls] == [A * K] * 5 and [b.shape[-1] for b in box] == [A * 4] * 5
    allc = torch.cat([c.reshape(-1) for c in cls])
    assert abs(float(allc.mean()) + 3.0) < 0.1 and abs(float(allc.std()) - 1.0) < 0.1
    out = ref.postprocess([c.numpy() for c in cls], [b.numpy() for b in box])
    assert out["boxes"].shape == (1, 100, 4) and out["classes"].dtype == np.int32
    assert int(out["is_valid"].sum()) == 100  # 5 x 1000 candidates above 0.05 -> 100 kept
    _check_layout(out["boxes"], out["scores"], out["classes"], out["is_valid"])
    _same_class_overlap_ok(out["boxes"], out["classes"], out["is_valid"])


# ------------------------------------------------------------- C4 (GPU)
def _gpu_head(model, batch):
    det = model.detector
    images = model.preprocess_image(batch)
    feats = model.neck(model.backbone(images.tensor))
    return det.head([feats[f] for f in det.in_features])


def _calibrated_gpu_model(dev, depth, batch):
    from detectron2_tensorflow_amd.utils.synthetic import calibrate_retinanet_head
    model = _model(depth).to(dev)
    with torch.no_grad():
        cls, box = _gpu_head(model, batch)
        calibrate_retinanet_head(model.detector.head, cls, box)
    return model


def _assert_post_matches_oracle(ref, cls, box, got):
    """Post-processing parity on identical head outputs: valid flags and class
    ids bit-exact, scores to 2e-7 relative (the sigmoid's expf), boxes within
    max(1e-4, 2 ulp)."""
    from test_gpu_ops import assert_boxes_close, assert_sigmoid_scores_close
    want = ref.postprocess([c.cpu().numpy() for c in cls], [b.cpu().numpy() for b in box])
    g = {k: v.cpu().numpy() for k, v in got.items()}
    np.testing.assert_array_equal(g["is_valid"], want["is_valid"])
    np.testing.assert_array_equal(g["classes"], want["classes"])
    assert_sigmoid_scores_close(g["scores"], want["scores"])
    for n in range(g["boxes"].shape[0]):
        assert_boxes_close(g["boxes"][n], want["boxes"][n])
    return want


@pytest.mark.gpu
def test_c4_retinanet_r50_640_vs_cpu_restatement(dev):
    import cpu_pipeline as cp
    rng = np.random.default_rng(5)
    img = rng.uniform(0, 255, (2, 640, 640, 3)).astype(F32)
    shapes = np.array([[640, 640], [600, 620]], np.int32)
    batch = {"image": torch.from_numpy(img).to(dev), "image_shape": torch.from_numpy(shapes).to(dev)}
    model = _calibrated_gpu_model(dev, 50, batch)
    with torch.no_grad():
        cls, box = _gpu_head(model, batch)
        out = model(batch)["instances"]
        post = model.detector.inference(cls, box)
    ref = cp.CPURetinaNet(model)
    # 1. the model's own forward == its head + post-processing
    for k, f in (("boxes", post.boxes), ("scores", post.get_field("scores")),
                 ("classes", post.get_field("pred_classes")), ("is_valid", post.get_field("is_valid"))):
        assert torch.equal(out[k], f), k
    # 2. post-processing on identical head outputs: bit-exact vs the oracle
    got = {"boxes": out["boxes"], "scores": out["scores"], "classes": out["classes"],
           "is_valid": out["is_valid"]}
    _assert_post_matches_oracle(ref, cls, box, got)
    # 3. head outputs vs the CPU restatement of backbone + FPN(P6P7) + tower
    with torch.no_grad():
        wcls, wbox = ref.head(ref.features(img))
    for g_, w_ in zip(list(cls) + list(box), list(wcls) + list(wbox)):
        err = (g_.cpu() - w_).abs().max().item()
        assert err <= 1e-3 * max(w_.abs().max().item(), 1.0), err
    # 4. end to end: detections of the whole GPU model vs the whole CPU restatement
    want = ref.postprocess([c.numpy() for c in wcls], [b.numpy() for b in wbox])
    g = {k: v.cpu().numpy() for k, v in got.items()}
    for n in range(2):
        wv, gv = want["is_valid"][n], g["is_valid"][n]
        hits = 0
        for b, c in zip(want["boxes"][n][wv], want["classes"][n][wv]):
            d = np.abs(g["boxes"][n][gv] - b).max(axis=1)
            hits += bool(((d < 1e-2) & (g["classes"][n][gv] == c)).any())
        assert hits >= 0.95 * wv.sum(), (n, hits, int(wv.sum()))
    _check_layout(g["boxes"], g["scores"], g["classes"], g["is_valid"])


@pytest.mark.gpu
def test_c4_retinanet_r101_1333x800_dense_anchors(dev):
    """C4 geometry: 800x1333 padded to 800x1344, p3..p7 = 100x168 ... 7x11,
    201,600 anchors/img x 80 classes (p3 alone 12.1 M scores).  Post-processing
    bit-exact vs the oracle on the GPU's own head outputs at full size;
    two runs identical; reference output layout."""
    import cpu_pipeline as cp
    g = torch.Generator(device="cpu").manual_seed(9)
    img = torch.rand(2, 800, 1333, 3, generator=g) * 255
    batch = {"image": img.to(dev), "image_shape": torch.tensor([[800, 1333], [800, 1333]], device=dev)}
    model = _calibrated_gpu_model(dev, 101, batch)
    old = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True  # any torch fallback conv (MIOpen): no atomic split-K
    try:
        with torch.no_grad():
            cls, box = _gpu_head(model, batch)
            a = model(batch)["instances"]
            b = model(batch)["instances"]
    finally:
        torch.backends.cudnn.deterministic = old
    assert [tuple(c.shape[1:3]) for c in cls] == [(100, 168), (50, 84), (25, 42), (13, 21), (7, 11)]
    assert sum(c.shape[1] * c.shape[2] * 9 for c in cls) == 201600
    for k in a:
        assert torch.equal(a[k], b[k]), k
    ref = cp.CPURetinaNet(model)
    _assert_post_matches_oracle(ref, cls, box, a)
    h = {k: v.cpu().numpy() for k, v in a.items()}
    _check_layout(h["boxes"], h["scores"], h["classes"], h["is_valid"])
    _same_class_overlap_ok(h["boxes"], h["classes"], h["is_valid"])
    assert int(h["is_valid"].sum()) == 200


def _train_cfg(depth=50):
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    cfg = get_cfg()
    name = "retinanet_R_50_FPN_1x.yaml" if depth == 50 else "retinanet_R_101_FPN_3x.yaml"
    cfg.merge_from_file(os.path.join(ROOT, "configs", "COCO-Detection", name))
    finalize(cfg, True, 1, CM)
    return cfg


@pytest.mark.gpu
@pytest.mark.parametrize("gamma", [None, 0.0])
def test_retina_fused_loss_matches_dense_formulation(dev, gamma):
    """d2mi_retina_loss_fwd / _bwd (csrc/retina_loss.hip) against the tensor
    formulation of RetinaNet.losses (retinanet.py:147-210: one-hot targets,
    sigmoid_focal_loss "sum" over the valid anchors, smooth-L1 "sum" over the
    foreground ones) on the same matcher output: both sums to 1e-5 relative,
    the gradients of every level's logits and deltas to 1e-5 relative (the
    kernel's float sequence differs from torch's composite ops)."""
    from detectron2_tensorflow_amd.layers import ShapeSpec, ops
    from detectron2_tensorflow_amd.modeling.matcher import match_boxes
    from detectron2_tensorflow_amd.modeling.single_stage_heads.retinanet import RetinaNetHead
    cfg = _train_cfg()
    feats = cfg.MODEL.SINGLE_STAGE_HEAD.IN_FEATURES
    strides = {f: 2 ** int(f[1:]) for f in feats}
    head = RetinaNetHead(cfg, {f: ShapeSpec(channels=16, stride=strides[f]) for f in feats}).to(dev)
    if gamma is not None:  # plain BCE (q^(gamma-1) at a saturated logit)
        head.focal_loss_gamma = gamma
    rng = np.random.default_rng(1)
    N, H, W, G, K = 2, 256, 320, 7, 80
    A = head.anchor_generator.num_cell_anchors[0]
    grids = [(-(-H // strides[f]), -(-W // strides[f])) for f in feats]
    fake = [torch.empty(N, h, w, 1, device=dev) for h, w in grids]
    anchors = head._all_anchors(fake)
    cy, cx = rng.uniform(0, H, (N, G)), rng.uniform(0, W, (N, G))
    hh, ww = rng.uniform(16, 200, (N, G)), rng.uniform(16, 200, (N, G))
    gt = np.stack([cy - hh / 2, cx - ww / 2, cy + hh / 2, cx + ww / 2], -1).astype(F32)
    valid = np.ones((N, G), bool)
    valid[1, 4:] = False
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    gcls = t(rng.integers(0, K, (N, G)))
    m, lab = match_boxes(head.matcher, t(gt), t(valid), anchors)
    assert int((lab == 1).sum()) > 10 and int((lab == -1).sum()) > 10
    cls = [rng.normal(-3, 1.5, (N, h, w, A * K)).astype(F32) for h, w in grids]
    cls[0][..., :7] = -30.0  # saturated: q = 1 - p_t rounds to 0 on the negatives
    cls = [t(c).requires_grad_() for c in cls]
    box = [t(rng.normal(0, 0.3, (N, h, w, A * 4)).astype(F32)).requires_grad_() for h, w in grids]
    got = ops.retina_loss(cls, box, anchors, t(gt), gcls, m, lab, K, A, head.focal_loss_alpha,
                          head.focal_loss_gamma, head.smooth_l1_loss_beta,
                          head.box2box_transform.weights)
    gg = torch.autograd.grad(got[0] * 0.7 + got[1] * 1.3, cls + box)
    want = head._losses_dense(cls, box, anchors, t(gt), gcls, m, lab)
    gw = torch.autograd.grad(want[0] * 0.7 + want[1] * 1.3, cls + box)
    for a, b in zip(got, want):
        assert float(a) == pytest.approx(float(b), rel=1e-5)
    for a, b in zip(gg, gw):
        assert torch.isfinite(a).all()
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7)


@pytest.mark.gpu
def test_retinanet_odd_class_count_takes_the_tensor_losses(dev):
    """NUM_CLASSES % 4 != 0: the fused kernels read float4 class
    quads, so such a head takes the tensor formulation on the GPU instead of
    raising (both losses finite)."""
    from detectron2_tensorflow_amd.layers import ShapeSpec
    from detectron2_tensorflow_amd.modeling.single_stage_heads.retinanet import RetinaNetHead
    cfg = _train_cfg()
    cfg.defrost()
    cfg.MODEL.SINGLE_STAGE_HEAD.NUM_CLASSES = 3
    cfg.freeze()
    feats = cfg.MODEL.SINGLE_STAGE_HEAD.IN_FEATURES
    strides = {f: 2 ** int(f[1:]) for f in feats}
    torch.manual_seed(0)
    head = RetinaNetHead(cfg, {f: ShapeSpec(channels=16, stride=strides[f]) for f in feats}).to(dev)
    head.train()
    assert head.num_classes == 3
    H, W = 128, 160
    fm = [torch.randn(1, -(-H // strides[f]), -(-W // strides[f]), 16, device=dev) for f in feats]
    box_cls, box_delta = head.head(fm)
    gt = {"gt_boxes": torch.tensor([[[10., 12., 90., 120.], [40., 50., 70., 100.]]], device=dev),
          "gt_classes": torch.tensor([[1, 2]], device=dev),
          "is_valid": torch.ones(1, 2, dtype=torch.bool, device=dev)}
    out = head.losses(fm, box_cls, box_delta, gt)
    assert torch.isfinite(out["loss_cls"]) and torch.isfinite(out["loss_box_reg"])


@pytest.mark.gpu
def test_retinanet_training_steps(dev):
    """RetinaNet R50-FPN training through the Trainer at 256x320 (the
    focal-loss path of retinanet.py:147-283 on the fused HIP matcher and
    loss): every trainable parameter gets a finite gradient, the loss
    normaliser follows its EMA of the foreground count on the device, and
    over-fitting one batch lowers the loss; the GPU losses of the first step
    equal the tensor formulation's on the same weights."""
    from detectron2_tensorflow_amd.engine import Trainer
    from detectron2_tensorflow_amd.modeling import build_model
    from detectron2_tensorflow_amd.modeling.single_stage_heads import retinanet as rmod
    from detectron2_tensorflow_amd.utils.synthetic import synthetic_train_batch
    cfg = _train_cfg()
    cfg.defrost()
    cfg.SOLVER.BASE_LR = 0.005
    cfg.SOLVER.WARMUP_ITERS = 0
    cfg.freeze()
    torch.manual_seed(0)
    model = build_model(cfg).to(dev).train()
    batch = synthetic_train_batch(2, 256, 320, 4, dev)
    losses = {}
    for fused in (False, True):
        rmod.FUSED_LOSSES = fused
        try:
            model.detector.loss_normalizer.fill_(100.0)
            model.zero_grad(set_to_none=True)
            losses[fused] = model(batch)
            if fused:
                sum(losses[fused].values()).backward()
        finally:
            rmod.FUSED_LOSSES = True
    assert set(losses[True]) == {"loss_cls", "loss_box_reg"}
    for k in losses[True]:
        assert float(losses[True][k]) == pytest.approx(float(losses[False][k]), rel=1e-5), k
    bad = [n for n, p in model.named_parameters()
           if p.requires_grad and (p.grad is None or not torch.isfinite(p.grad).all())]
    assert not bad, bad[:5]
    model.detector.loss_normalizer.fill_(100.0)
    tr = Trainer(cfg, model)
    hist, norms = [], []
    for _ in range(12):
        out = tr.step(batch)
        norms.append(float(model.detector.loss_normalizer))
        hist.append(float(out["total_loss"]) * norms[-1])  # the raw sums (the EMA drifts)
    assert all(np.isfinite(hist)), hist
    # EMA towards the (constant) foreground count: monotone, strictly moving
    d = np.diff(norms)
    assert (d <= 0).all() or (d >= 0).all(), norms
    assert abs(norms[-1] - 100.0) > 1.0
    assert np.mean(hist[-3:]) < 0.9 * np.mean(hist[:3]), hist
    from detectron2_tensorflow_amd import _C
    _C.raise_on_errors(dev)
