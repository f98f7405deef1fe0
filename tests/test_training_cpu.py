"""CPU tests of the training-side host logic (no GPU): batched Matcher /
subsample / pairwise IoU, the RPN and Fast R-CNN loss glue against the
per-image oracle restatement, the LR schedule, the Momentum-SGD update, and
the bucketed all-reduce over gloo with world_size 2."""
import os
import socket

import numpy as np
import pytest
import torch

import training as otrain
from detectron2_tensorflow_amd.modeling.matcher import Matcher, pairwise_iou, subsample_labels


def rand_boxes(rng, n, H=200, W=300, smin=4, smax=120):
    cy, cx = rng.uniform(0, H, n), rng.uniform(0, W, n)
    h, w = rng.uniform(smin, smax, n), rng.uniform(smin, smax, n)
    return np.stack([cy - h / 2, cx - w / 2, cy + h / 2, cx + w / 2], 1).astype(np.float32)


def test_pairwise_iou_matches_oracle():
    rng = np.random.default_rng(0)
    a, b = rand_boxes(rng, 7), rand_boxes(rng, 50)
    b[3] = 0  # zero-area: union may be 0 -> 0
    a[2] = 0
    got = pairwise_iou(torch.from_numpy(a)[None], torch.from_numpy(b)[None])[0].numpy()
    np.testing.assert_array_equal(got, otrain.pairwise_iou(a, b))


@pytest.mark.parametrize("seed", range(4))
def test_matcher_matches_oracle_per_image(seed):
    rng = np.random.default_rng(seed)
    N, G, P = 3, 6, 300
    gt = rand_boxes(rng, N * G).reshape(N, G, 4)
    pr = rand_boxes(rng, N * P).reshape(N, P, 4)
    pr[:, :5] = gt[:, :5] + 0.0  # exact hits and ties
    valid = rng.random((N, G)) < 0.8
    valid[2] = False  # an image without valid GT: all background
    crowd = rng.random((N, G)) < 0.2
    m = Matcher([0.3, 0.7], [0, -1, 1], allow_low_quality_matches=True)
    q = pairwise_iou(torch.from_numpy(gt), torch.from_numpy(pr))
    crowd_t = torch.from_numpy(crowd)
    cq = torch.where(crowd_t[..., None], q, torch.zeros_like(q))
    matches, labels = m(q, torch.from_numpy(valid & ~crowd), cq)
    for i in range(N):
        v = valid[i] & ~crowd[i]
        om, ol = otrain.matcher(otrain.pairwise_iou(gt[i][v], pr[i]), [0.3, 0.7], [0, -1, 1], True,
                                otrain.pairwise_iou(gt[i][crowd[i]], pr[i]))
        np.testing.assert_array_equal(labels[i].numpy(), ol)
        if v.any():
            # match indices are into the valid subset in the reference
            np.testing.assert_array_equal(np.nonzero(v)[0][om][ol == 1], matches[i].numpy()[ol == 1])


def test_subsample_labels_counts_and_membership():
    g = torch.Generator().manual_seed(0)
    labels = torch.full((4, 5000), -1, dtype=torch.int64)
    labels[0, :300] = 1
    labels[0, 300:4000] = 0
    labels[1, :20] = 3
    labels[1, 20:60] = 0       # too few negatives: 20 + 40
    labels[2, 100:2000] = 0    # no positives: all negatives
    labels[3, :] = -1          # nothing to sample
    pos, neg = subsample_labels(labels, 256, 0.5, 0, generator=g)
    np.testing.assert_array_equal(pos.sum(1).numpy(), [128, 20, 0, 0])
    np.testing.assert_array_equal(neg.sum(1).numpy(), [128, 40, 256, 0])
    assert not (pos & neg).any()
    assert ((labels > 0) | ~pos).all() and ((labels == 0) | ~neg).all()


def test_lr_schedule_warmup_and_steps():
    from detectron2_tensorflow_amd.config import get_cfg
    from detectron2_tensorflow_amd.solver import build_learning_rate
    cfg = get_cfg()
    cfg.SOLVER.BASE_LR, cfg.SOLVER.STEPS, cfg.SOLVER.GAMMA = 0.02, (100, 200), 0.1
    cfg.SOLVER.WARMUP_ITERS, cfg.SOLVER.WARMUP_FACTOR = 10, 0.001
    cfg.SOLVER.IMS_PER_BATCH, cfg.SOLVER.IMS_PER_BATCH_BASE = 32, 16
    lr = build_learning_rate(cfg)
    # auto-scale: boundaries / 2, values * 2
    assert lr(0) == pytest.approx(0.04 * 0.001)
    assert lr(5) == pytest.approx(0.04 * (0.001 * 0.5 + 0.5))
    assert lr(10) == pytest.approx(0.04)
    assert lr(50) == pytest.approx(0.04)      # piecewise_constant: <= boundary keeps value
    assert lr(51) == pytest.approx(0.004)
    assert lr(101) == pytest.approx(0.0004)


def test_momentum_sgd_matches_reference_update():
    from detectron2_tensorflow_amd.solver import MomentumSGD
    rng = np.random.default_rng(1)
    shapes = [(3, 3, 4, 8), (8,), (16,)]
    ps = [torch.nn.Parameter(torch.from_numpy(rng.standard_normal(s).astype(np.float32)))
          for s in shapes]
    groups = [{"params": [ps[0]], "weight_decay": 1e-4}, {"params": [ps[1]], "weight_decay": 1e-4},
              {"params": [ps[2]], "weight_decay": 0.0}]
    opt = MomentumSGD(groups, momentum=0.9, clip_norm=10.0)
    ref_p = [p.detach().numpy().astype(np.float64) for p in ps]
    ref_a = [np.zeros_like(p) for p in ref_p]
    for step in range(3):
        gs = [rng.standard_normal(s).astype(np.float32) * (30 if i == 0 else 0.1)
              for i, s in enumerate(shapes)]
        for p, g in zip(ps, gs):
            p.grad = torch.from_numpy(g.copy())
        opt.step(0.01)
        ref_p, ref_a = otrain.sgd_step(ref_p, gs, ref_a, 0.01, 0.9, [1e-4, 1e-4, 0.0], 10.0)
        for p, r in zip(ps, ref_p):
            np.testing.assert_allclose(p.detach().numpy(), r, rtol=1e-5, atol=1e-6)


def _small_cfg():
    from detectron2_tensorflow_amd.config import get_cfg
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(os.path.dirname(__file__), "..", "configs",
                                     "COCO-InstanceSegmentation", "mask_rcnn_R_50_FPN_1x.yaml"))
    return cfg


def test_rpn_losses_match_oracle_when_everything_is_sampled():
    """With fewer candidates than the sampling caps, subsample_labels takes all of
    them and the reference becomes deterministic: compare the dense batched loss
    with the per-image restatement."""
    from detectron2_tensorflow_amd.modeling.proposal_generator.rpn import RPN
    from detectron2_tensorflow_amd.layers import ShapeSpec
    from detectron2_tensorflow_amd.structures import ImageList
    import oracle
    cfg = _small_cfg()
    cfg.MODEL.RPN.IN_FEATURES = ["p3"]
    cfg.MODEL.ANCHOR_GENERATOR.SIZES = [[32, 64]]
    cfg.MODEL.ANCHOR_GENERATOR.ASPECT_RATIOS = [[0.5, 1.0]]
    rpn = RPN(cfg, {"p3": ShapeSpec(channels=8, stride=8)})
    rng = np.random.default_rng(3)
    N, H, W, G = 2, 6, 7, 4
    cell = oracle.generate_cell_anchors([32, 64], [0.5, 1.0])
    anchors = oracle.grid_anchors(H, W, 8, cell)           # 168 anchors < 256
    A = anchors.shape[0] // (H * W)
    feats = [torch.zeros(N, H, W, 8)]
    rpn._anchors, rpn._anchor_key = torch.from_numpy(anchors), \
        ((H, W), str(feats[0].device))
    gt = rand_boxes(rng, N * G, H=48, W=56, smin=16, smax=60).reshape(N, G, 4)
    valid = np.array([[1, 1, 1, 0], [1, 0, 1, 1]], bool)
    crowd = np.array([[0, 0, 1, 0], [0, 0, 0, 0]], bool)
    logits = [torch.from_numpy(rng.standard_normal((N, H, W, A)).astype(np.float32))]
    deltas = [torch.from_numpy(rng.standard_normal((N, H, W, 4 * A)).astype(np.float32) * 0.1)]
    images = ImageList(torch.zeros(N, 48, 56, 3), torch.tensor([[48, 56]] * N, dtype=torch.int32))
    targets = {"gt_boxes": torch.from_numpy(gt), "is_valid": torch.from_numpy(valid),
               "gt_is_crowd": torch.from_numpy(crowd)}
    losses = rpn.losses(images, feats, logits, deltas, targets)
    labs, dels = [], []
    for i in range(N):
        lab, d = otrain.rpn_targets(anchors, gt[i], valid[i], crowd[i], (1, 1, 1, 1), [0.3, 0.7],
                                    [0, -1, 1])
        assert (lab == 1).sum() <= 128
        labs.append(lab)
        dels.append(d)
    cls, loc = otrain.rpn_losses(np.concatenate(labs), np.concatenate(dels),
                                 logits[0].numpy().reshape(-1), deltas[0].numpy().reshape(-1, 4), N, 256)
    assert losses["loss_rpn_cls"].item() == pytest.approx(cls, rel=1e-5)
    assert losses["loss_rpn_loc"].item() == pytest.approx(loc, rel=1e-5)


def test_roi_label_and_sample_and_box_losses_match_oracle():
    from detectron2_tensorflow_amd.modeling.roi_heads.fast_rcnn import fast_rcnn_losses
    from detectron2_tensorflow_amd.modeling.roi_heads.roi_heads import ROIHeads
    from detectron2_tensorflow_amd.modeling.box_regression import Box2BoxTransform
    from detectron2_tensorflow_amd.structures import BoxList
    from detectron2_tensorflow_amd.layers import ShapeSpec
    cfg = _small_cfg()
    K = 5
    cfg.MODEL.ROI_HEADS.NUM_CLASSES = K
    heads = ROIHeads(cfg, {f"p{i}": ShapeSpec(channels=8, stride=2 ** i) for i in range(2, 6)})
    rng = np.random.default_rng(5)
    N, P, G = 2, 120, 5
    gt = rand_boxes(rng, N * G).reshape(N, G, 4)
    props = rand_boxes(rng, N * P).reshape(N, P, 4)
    props[:, :40] = gt[:, rng.integers(0, G, 40)] + rng.normal(0, 4, (N, 40, 4)).astype(np.float32)
    pvalid = np.ones((N, P), bool)
    pvalid[1, 100:] = False
    gvalid = np.array([[1, 1, 1, 1, 0], [1, 1, 0, 1, 1]], bool)
    crowd = np.zeros((N, G), bool)
    crowd[0, 3] = True
    diff = np.zeros((N, G), bool)
    diff[1, 4] = True
    gcls = rng.integers(0, K, (N, G))
    pl = BoxList(torch.from_numpy(props))
    pl.add_field("is_valid", torch.from_numpy(pvalid))
    targets = {"gt_boxes": torch.from_numpy(gt), "gt_classes": torch.from_numpy(gcls),
               "is_valid": torch.from_numpy(gvalid), "gt_is_crowd": torch.from_numpy(crowd),
               "gt_difficult": torch.from_numpy(diff)}
    s = heads.label_and_sample_proposals(pl, targets)
    S = heads.batch_size_per_image
    R_total = int(s["is_valid"].sum())
    logits = torch.from_numpy(rng.standard_normal((N * S, K + 1)).astype(np.float32))
    deltas = torch.from_numpy(rng.standard_normal((N * S, 4 * K)).astype(np.float32) * 0.1)
    got = fast_rcnn_losses(logits, deltas, s["boxes"].reshape(-1, 4), s["gt_classes"].reshape(-1),
                           s["gt_boxes"].reshape(-1, 4), s["is_valid"].reshape(-1),
                           Box2BoxTransform((10, 10, 5, 5)), 0.0)
    rows, ocls, ogt, oprops = [], [], [], []
    for i in range(N):
        pr, cl, mg = otrain.label_proposals(props[i], pvalid[i], gt[i], gcls[i], gvalid[i], crowd[i],
                                            diff[i], K, 0.5)
        nfg = ((cl >= 0) & (cl < K)).sum()
        assert nfg <= 128 and (cl >= 0).sum() <= S
        # dense layout: fg first then bg, each in proposal order (all sampled)
        sv = s["is_valid"][i].numpy()
        scl = s["gt_classes"][i].numpy()[sv]
        order = np.concatenate([np.nonzero((cl >= 0) & (cl < K))[0], np.nonzero(cl == K)[0]])
        np.testing.assert_array_equal(np.sort(scl[:nfg]), np.sort(cl[order[:nfg]]))
        np.testing.assert_array_equal(s["boxes"][i].numpy()[sv], pr[order])
        np.testing.assert_array_equal(scl, cl[order])
        fg = scl < K
        np.testing.assert_array_equal(s["gt_boxes"][i].numpy()[sv][fg], mg[order][fg])
        rows.append(np.nonzero(sv)[0] + i * S)
        ocls.append(cl[order])
        ogt.append(mg[order])
        oprops.append(pr[order])
    rows = np.concatenate(rows)
    assert len(rows) == R_total
    lc, lb = otrain.fast_rcnn_losses(logits.numpy()[rows], deltas.numpy()[rows],
                                     np.concatenate(oprops), np.concatenate(ocls),
                                     np.concatenate(ogt), (10, 10, 5, 5))
    assert got["loss_cls"].item() == pytest.approx(lc, rel=1e-5)
    assert got["loss_box_reg"].item() == pytest.approx(lb, rel=1e-5)


# --------------------------------------------------------------- gloo, world 2
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _toy_model(seed):
    torch.manual_seed(seed)
    return torch.nn.Sequential(torch.nn.Linear(16, 64), torch.nn.ReLU(), torch.nn.Linear(64, 64),
                               torch.nn.ReLU(), torch.nn.Linear(64, 3))


def _batch(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(8, 16, generator=g), torch.randn(8, 3, generator=g)


def _dp_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from detectron2_tensorflow_amd.engine import BucketedAllReduce, broadcast_parameters
    from detectron2_tensorflow_amd.solver import MomentumSGD
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = _toy_model(seed=rank)  # different init per rank: broadcast must fix it
    broadcast_parameters(model)
    params = list(model.parameters())
    opt = MomentumSGD([{"params": params, "weight_decay": 1e-4}], 0.9, 10.0)
    red = BucketedAllReduce(params, bucket_bytes=4096)  # several buckets
    assert len(red.buckets) > 2
    for it in range(3):
        opt.zero_grad()
        red.reset()
        x, y = _batch(rank * 10 + it)
        torch.nn.functional.mse_loss(model(x), y).backward()
        red.finish()
        opt.step(0.05)
    torch.save({k: v.detach().clone() for k, v in model.state_dict().items()},
               os.path.join(out_dir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def test_bucketed_allreduce_gloo_world2_matches_single_process(tmp_path):
    import torch.multiprocessing as mp
    from detectron2_tensorflow_amd.solver import MomentumSGD
    world = 2
    mp.spawn(_dp_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    for k in r0:
        torch.testing.assert_close(r0[k], r1[k], rtol=0, atol=0)
    # single process, gradient = mean of the two shards' gradients
    model = _toy_model(seed=0)
    params = list(model.parameters())
    opt = MomentumSGD([{"params": params, "weight_decay": 1e-4}], 0.9, 10.0)
    for it in range(3):
        grads = []
        for rank in range(world):
            model.zero_grad()
            x, y = _batch(rank * 10 + it)
            torch.nn.functional.mse_loss(model(x), y).backward()
            grads.append([p.grad.clone() for p in params])
        for i, p in enumerate(params):
            p.grad = (grads[0][i] + grads[1][i]) / world
        opt.step(0.05)
    for k, v in model.state_dict().items():
        torch.testing.assert_close(r0[k], v, rtol=1e-5, atol=1e-6)


class _SharedBranchModel(torch.nn.Module):
    """A head shared across "levels" (used 3 times per forward, as the RPN head
    over p2..p6) and a branch that only runs when its input is non-empty (as
    a mask head on a rank with no foreground)."""

    def __init__(self, seed):
        super().__init__()
        torch.manual_seed(seed)
        self.stem = torch.nn.Linear(16, 32)
        self.shared = torch.nn.Linear(32, 32)
        self.branch = torch.nn.Linear(32, 3)
        self.out = torch.nn.Linear(32, 3)

    def forward(self, x, use_branch):
        h = torch.relu(self.stem(x))
        y = 0
        for s in (1.0, 0.5, 0.25):  # one parameter, three uses
            y = y + self.out(torch.relu(self.shared(h * s)))
        if use_branch:
            y = y + self.branch(h)
        return y


def _dp_shared_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from detectron2_tensorflow_amd.engine import BucketedAllReduce, broadcast_parameters
    from detectron2_tensorflow_amd.solver import MomentumSGD
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = _SharedBranchModel(seed=rank)
    broadcast_parameters(model)
    params = list(model.parameters())
    opt = MomentumSGD([{"params": params, "weight_decay": 0.0}], 0.9, 0.0)
    red = BucketedAllReduce(params, bucket_bytes=2048)  # the branch gets a bucket of its own
    for it in range(3):
        opt.zero_grad()
        red.reset()
        x, y = _batch(rank * 10 + it)
        # rank 1 never runs the branch: its .grad stays None there, and
        # finish() must contribute zeros for it (same collective sequence)
        torch.nn.functional.mse_loss(model(x, use_branch=(rank == 0)), y).backward()
        red.finish()
        opt.step(0.05)
    torch.save({k: v.detach().clone() for k, v in model.state_dict().items()},
               os.path.join(out_dir, f"shared{rank}.pt"))
    dist.destroy_process_group()


def test_bucketed_allreduce_shared_and_rank_local_params(tmp_path):
    """engine/reducer.py with a parameter used several times per forward (its
    post-accumulate hook fires once, on the summed gradient) and a parameter
    that gets no gradient on one rank only (the finish() zero fill): replicas
    stay bit-identical and equal the single-process mean-gradient update."""
    import torch.multiprocessing as mp
    from detectron2_tensorflow_amd.solver import MomentumSGD
    world = 2
    mp.spawn(_dp_shared_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0 = torch.load(tmp_path / "shared0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "shared1.pt", weights_only=True)
    for k in r0:
        torch.testing.assert_close(r0[k], r1[k], rtol=0, atol=0)
    model = _SharedBranchModel(seed=0)
    params = list(model.parameters())
    opt = MomentumSGD([{"params": params, "weight_decay": 0.0}], 0.9, 0.0)
    for it in range(3):
        grads = []
        for rank in range(world):
            model.zero_grad(set_to_none=True)
            x, y = _batch(rank * 10 + it)
            torch.nn.functional.mse_loss(model(x, use_branch=(rank == 0)), y).backward()
            grads.append([p.grad.clone() if p.grad is not None else torch.zeros_like(p)
                          for p in params])
        for i, p in enumerate(params):
            p.grad = (grads[0][i] + grads[1][i]) / world
        opt.step(0.05)
    for k, v in model.state_dict().items():
        torch.testing.assert_close(r0[k], v, rtol=1e-5, atol=1e-6)
    assert not torch.equal(r0["branch.weight"], _SharedBranchModel(seed=0).branch.weight)


def test_cpu_training_step_restatement_runs_and_updates():
    """oracle/cpu_train.py (bench.py's training cpu_baseline): one step on a tiny
    image gives finite losses and moves the trainable weights only."""
    import cpu_train
    from detectron2_tensorflow_amd.config import finalize
    from detectron2_tensorflow_amd.modeling import build_model
    from detectron2_tensorflow_amd.utils.synthetic import synthetic_train_batch
    cfg = _small_cfg()
    cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT = "raw"
    finalize(cfg, True, 1, {"num_thing_classes": 80, "num_stuff_classes": 53,
                            "stuff_ignore_value": 0})
    torch.manual_seed(0)
    model = build_model(cfg)
    step = cpu_train.CPUTrainStep(model, cfg)
    b = synthetic_train_batch(1, 128, 160, 0, torch.device("cpu"), sqrt_area=(16.0, 96.0))
    w_tr = step.m.roi_heads.box_head.fcs[0].weights.detach().clone()
    w_fz = step.m.backbone.stem.conv1.weights.detach().clone()
    losses = step.step(b["image"].numpy(), b["image_shape"].numpy(), b["instances"], threads=4)
    assert set(losses) == {"loss_rpn_cls", "loss_rpn_loc", "loss_cls", "loss_box_reg", "loss_mask"}
    assert all(np.isfinite(v) for v in losses.values()), losses
    assert not torch.equal(w_tr, step.m.roi_heads.box_head.fcs[0].weights.detach())
    assert torch.equal(w_fz, step.m.backbone.stem.conv1.weights.detach())


def test_cell_anchor_host_cache_follows_values():
    """ops._cell_host_array (the host copy of the cell anchors handed to the
    fused proposal / RetinaNet decoders) must follow the anchors' VALUES:
    models with different anchor sizes built and freed in one process (tensors
    at reused addresses), and in-place edits, never see a stale copy."""
    from detectron2_tensorflow_amd.layers import ops
    from detectron2_tensorflow_amd.modeling.anchor_generator import generate_cell_anchors
    for i in range(40):
        sizes = (32 * (1 + i % 3),)
        cells = [generate_cell_anchors(sizes, (0.5, 1, 2))]
        arr, n = ops._cell_host_array(cells)
        want = torch.as_tensor(cells[0], dtype=torch.float32).reshape(-1).tolist()
        assert n == len(want) and list(arr)[:n] == want
        del cells, arr
    c = generate_cell_anchors((64,), (1,))
    ops._cell_host_array([c])
    c.mul_(2)  # in place: the version counter moves, the copy is refreshed
    arr, n = ops._cell_host_array([c])
    assert list(arr)[:n] == c.reshape(-1).tolist()


def test_trainer_loss_terms_cast_and_reject():
    """Trainer._loss_terms: mixed float dtypes and Python numbers are summed as
    f32 scalars; a non-scalar or integer loss raises naming its key."""
    from detectron2_tensorflow_amd.engine.trainer import Trainer
    t = Trainer._loss_terms({"a": torch.tensor(1.5), "b": torch.tensor(2.0, dtype=torch.float64),
                             "c": 0.25, "d": torch.tensor([3.0])})
    assert all(x.dtype == torch.float32 and x.dim() == 0 for x in t)
    assert float(torch.stack(t).sum()) == 6.75
    with pytest.raises(TypeError, match="'bad'"):
        Trainer._loss_terms({"a": torch.tensor(1.0), "bad": torch.ones(2)})
    with pytest.raises(TypeError, match="'n'"):
        Trainer._loss_terms({"n": torch.tensor(3)})


def test_retinanet_dense_losses_match_oracle():
    """RetinaNetHead's tensor formulation of the training losses (the GPU
    kernel's reference in tests/test_retinanet.py) on the CPU Matcher, against
    the per-image restatement of get_ground_truth + losses
    (retinanet.py:147-283): targets, focal loss, smooth-L1, normaliser EMA."""
    import oracle
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    from detectron2_tensorflow_amd.layers import ShapeSpec
    from detectron2_tensorflow_amd.modeling.matcher import match_boxes
    from detectron2_tensorflow_amd.modeling.single_stage_heads.retinanet import RetinaNetHead
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(root, "configs", "COCO-Detection", "retinanet_R_50_FPN_1x.yaml"))
    cfg.MODEL.SINGLE_STAGE_HEAD.NUM_CLASSES = 8
    finalize(cfg, True, 1, {"num_thing_classes": 8, "num_stuff_classes": 0, "stuff_ignore_value": 0})
    feats = cfg.MODEL.SINGLE_STAGE_HEAD.IN_FEATURES
    strides = {f: 2 ** int(f[1:]) for f in feats}
    head = RetinaNetHead(cfg, {f: ShapeSpec(channels=16, stride=strides[f]) for f in feats})
    rng = np.random.default_rng(0)
    N, H, W, G, K = 2, 64, 96, 5, 8
    A = head.anchor_generator.num_cell_anchors[0]
    grids = [(-(-H // strides[f]), -(-W // strides[f])) for f in feats]
    anchors = np.concatenate([oracle.grid_anchors(h, w, strides[f], c.numpy())
                              for (h, w), f, c in zip(grids, feats, head.anchor_generator.cell_anchors)])
    gt = np.stack([rand_boxes(rng, G, H, W, 8, 60) for _ in range(N)])
    valid = np.array([[1, 1, 1, 0, 1], [1, 0, 0, 0, 0]], bool)
    gcls = rng.integers(0, K, (N, G))
    cls = [torch.from_numpy(rng.normal(0, 2, (N, h, w, A * K)).astype(np.float32)) for h, w in grids]
    box = [torch.from_numpy(rng.normal(0, 0.3, (N, h, w, A * 4)).astype(np.float32)) for h, w in grids]
    t = torch.from_numpy
    m, lab = match_boxes(head.matcher, t(gt), t(valid), t(anchors))
    cs, bs = head._losses_dense(cls, box, t(anchors), t(gt), t(gcls), m, lab)
    tc, td = zip(*[otrain.retinanet_targets(anchors, gt[i], gcls[i], valid[i], K,
                                                     head.box2box_transform.weights)
                   for i in range(N)])
    lg = np.concatenate([np.concatenate([c[i].numpy().reshape(-1, K) for c in cls]) for i in range(N)])
    dl = np.concatenate([np.concatenate([b[i].numpy().reshape(-1, 4) for b in box]) for i in range(N)])
    want_c, want_b, norm = otrain.retinanet_losses(
        np.concatenate(tc), np.concatenate(td), lg, dl, K, head.focal_loss_alpha,
        head.focal_loss_gamma, head.smooth_l1_loss_beta, 100.0)
    assert (np.concatenate(tc) >= 0).sum() > 0 and (np.concatenate(tc) < K).any()
    assert float(cs) / norm == pytest.approx(want_c, rel=1e-5)
    assert float(bs) / norm == pytest.approx(want_b, rel=1e-5)


def _solo_batch(seed, N=2, G=6, H=128, W=160):
    """Dense SOLOv2 targets: boxes across the scale ranges, box-filled masks
    at the padded image size, an invalid GT and a duplicated GT (two GT of one
    level claiming the same cells)."""
    rng = np.random.default_rng(seed)
    s = np.exp(rng.uniform(np.log(12), np.log(150), (N, G)))
    r = np.exp(rng.uniform(np.log(0.5), np.log(2.0), (N, G)))
    h, w = s * np.sqrt(r), s / np.sqrt(r)
    cy, cx = rng.uniform(0, H, (N, G)), rng.uniform(0, W, (N, G))
    boxes = np.stack([np.clip(cy - h / 2, 0, H - 4), np.clip(cx - w / 2, 0, W - 4),
                      np.clip(cy + h / 2, 4, H), np.clip(cx + w / 2, 4, W)], -1)
    boxes = np.round(boxes).astype(np.float32)
    boxes[..., 2] = np.maximum(boxes[..., 2], boxes[..., 0] + 4)
    boxes[..., 3] = np.maximum(boxes[..., 3], boxes[..., 1] + 4)
    boxes[0, 1] = boxes[0, 0]  # a duplicate: same box, another class
    classes = rng.integers(0, 5, (N, G))
    valid = np.ones((N, G), bool)
    valid[1, -1] = False
    masks = np.zeros((N, G, H, W), np.uint8)
    for b in range(N):
        for g in range(G):
            y1, x1, y2, x2 = boxes[b, g].astype(int)
            masks[b, g, y1:y2, x1:x2] = 1
    return boxes, classes, valid, masks


@pytest.mark.parametrize("seed", range(3))
def test_solov2_targets_match_oracle(seed):
    from detectron2_tensorflow_amd.modeling.single_stage_heads.solo_v2 import solov2_targets
    boxes, classes, valid, masks = _solo_batch(seed)
    grids, ranges = [40, 36, 24, 16, 12], [(1, 96), (48, 192), (96, 384), (192, 768), (384, 2048)]
    want = otrain.solov2_targets(boxes, classes, valid, masks, (32, 40), grids, ranges, 0.2)
    got = solov2_targets(torch.from_numpy(boxes), torch.from_numpy(classes),
                         torch.from_numpy(valid), torch.from_numpy(masks), (32, 40), grids, ranges,
                         0.2)
    npos = 0
    for (wc, wp, wm), (gc, gp, gm) in zip(want, got):
        np.testing.assert_array_equal(gc.numpy(), wc)
        np.testing.assert_array_equal(gp.numpy(), wp)
        np.testing.assert_array_equal(gm.numpy(), wm)
        npos += len(wp)
    assert npos > 10


def test_solov2_losses_match_oracle():
    from types import SimpleNamespace

    from detectron2_tensorflow_amd.modeling.single_stage_heads.solo_v2 import MaskKernelBranch
    boxes, classes, valid, masks = _solo_batch(7)
    grids, ranges = [40, 36, 24, 16, 12], [(1, 96), (48, 192), (96, 384), (192, 768), (384, 2048)]
    N, K, E, Hm, Wm = 2, 5, 8, 32, 40
    g = torch.Generator().manual_seed(0)
    pc = [torch.randn(N, S, S, K, generator=g) - 2 for S in grids]
    pk = [torch.randn(N, S, S, E, generator=g) * 0.3 for S in grids]
    mf = torch.randn(N, Hm, Wm, E, generator=g)
    me = SimpleNamespace(num_grids=grids, scale_ranges=ranges, sigma=0.2, num_classes=K,
                         focal_loss_alpha=0.25, focal_loss_gamma=2.0, ins_loss_weight=3.0)
    tg = {"gt_boxes": torch.from_numpy(boxes), "gt_classes": torch.from_numpy(classes),
          "is_valid": torch.from_numpy(valid), "gt_masks": torch.from_numpy(masks)}
    for t in pc + pk + [mf]:
        t.requires_grad_(True)
    got = MaskKernelBranch.losses(me, pc, pk, mf, tg)
    want_t = otrain.solov2_targets(boxes, classes, valid, masks, (Hm, Wm), grids, ranges, 0.2)
    ins, cls = otrain.solov2_losses([t.detach().numpy() for t in pc],
                                    [t.detach().numpy() for t in pk], mf.detach().numpy(), want_t,
                                    K, 0.25, 2.0, 3.0)
    np.testing.assert_allclose(float(got["loss_ins"].detach()), ins, rtol=1e-5)
    np.testing.assert_allclose(float(got["loss_cls"].detach()), cls, rtol=1e-5)
    (got["loss_ins"] + got["loss_cls"]).backward()
    assert all(t.grad is not None and torch.isfinite(t.grad).all() for t in pk[:2] + [mf])
