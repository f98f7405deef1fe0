"""GPU tests of the hipGraph-replayed training step (engine/graphed.py): the
graphed trainer's weights, momentum and losses equal the eager Trainer's bit
for bit -- after one replay, and over steps that change the mask branch's
row count, across an eager step in the middle (kernel timing), and with a new
batch object each step (copied into the captured inputs).

r4 removed these tests after the replays faulted; r5 found the cause (host
tables allocated inside the capture shared memory with captured temporaries:
utils/capture.py, tools/graph_audit.py) and restored them."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CATS = {"num_thing_classes": 80, "num_stuff_classes": 53, "stuff_ignore_value": 0}


def _model(dev):
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    from detectron2_tensorflow_amd.modeling import build_model
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, "configs", "COCO-InstanceSegmentation",
                                     "mask_rcnn_R_50_FPN_1x.yaml"))
    cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT = "raw"
    cfg.SOLVER.WARMUP_ITERS = 3  # the LR changes every step: read from the device
    finalize(cfg, True, 1, CATS)
    torch.manual_seed(0)
    return cfg, build_model(cfg).to(dev).train()


def test_graphed_step_one_replay_matches_eager_step(dev, monkeypatch):
    """Graph A + the B[R] graphs captured once, ONE replay: losses, weights and
    momentum bit-identical to Trainer.step on the same inputs."""
    from detectron2_tensorflow_amd.engine import Trainer
    from detectron2_tensorflow_amd.engine.graphed import GraphedTrainer
    from detectron2_tensorflow_amd.utils.synthetic import (calibrate_rcnn_scores,
                                                           synthetic_train_batch)
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    cfg, m_eager = _model(dev)
    _, m_graph = _model(dev)
    batch = synthetic_train_batch(2, 256, 320, 11, dev)
    calibrate_rcnn_scores(m_eager, batch)
    m_graph.load_state_dict(m_eager.state_dict())
    eager = Trainer(cfg, m_eager)
    graphed = GraphedTrainer(cfg, m_graph, warmup=1)
    for i in range(2):  # 0: the graphed trainer's eager warm-up; 1: capture + ONE replay
        torch.manual_seed(100 + i)
        le = eager.step(batch)
        torch.manual_seed(100 + i)
        lg = graphed.step(batch)
        torch.cuda.synchronize()
        assert set(le) == set(lg)
        for k in le:
            assert torch.equal(le[k].reshape(()), lg[k].reshape(())), (i, k, le[k], lg[k])
        for (n, pe), pg in zip(m_eager.named_parameters(), m_graph.parameters()):
            assert torch.equal(pe, pg), (i, n)
        for ae, ag in zip(eager.optimizer.accum, graphed.optimizer.accum):
            assert torch.equal(ae, ag), i
    assert graphed.replays == 1
    from detectron2_tensorflow_amd import _C
    _C.raise_on_errors(dev)


def _alternating_steps(dev, monkeypatch, height, width, steps, eager_at, seeds, num_gt=7):
    """Eager Trainer vs GraphedTrainer over ``steps`` steps on two batches
    that alternate (the second with fewer GT boxes: other foreground counts,
    so other mask-row counts and other B[R] graphs); step 0 is the graphed
    trainer's eager warm-up, step ``eager_at`` an eager step between replays,
    every other step a replay.  Losses, every weight and every momentum
    torch.equal after each step."""
    from detectron2_tensorflow_amd.engine import Trainer
    from detectron2_tensorflow_amd.engine.graphed import GraphedTrainer
    from detectron2_tensorflow_amd.utils.synthetic import (calibrate_rcnn_scores,
                                                           synthetic_train_batch)
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    cfg, m_eager = _model(dev)
    _, m_graph = _model(dev)
    batches = [synthetic_train_batch(2, height, width, s, dev, num_gt=num_gt) for s in seeds]
    batches[1]["instances"]["is_valid"][:, 2:] = False  # fewer GT: other mask row counts
    calibrate_rcnn_scores(m_eager, batches[0])  # (draws random logit scales: once)
    m_graph.load_state_dict(m_eager.state_dict())
    eager = Trainer(cfg, m_eager)
    graphed = GraphedTrainer(cfg, m_graph, warmup=1)
    heads = graphed.heads[0]
    rows = []
    # new batch objects each step for the graphed trainer: copied into the
    # captured inputs
    for i in range(steps):
        b = batches[i % 2]
        bg = {k: (v.clone() if torch.is_tensor(v) else {kk: vv.clone() for kk, vv in v.items()})
              for k, v in b.items()}
        torch.manual_seed(100 + i)
        le = eager.step(b)
        torch.manual_seed(100 + i)
        lg = graphed.eager_step(bg) if i == eager_at else graphed.step(bg)
        rows.append(heads.last_mask_rows)
        assert set(le) == set(lg)
        for k in le:
            assert torch.equal(le[k].reshape(()), lg[k].reshape(())), (i, k, le[k], lg[k])
        for (n, pe), pg in zip(m_eager.named_parameters(), m_graph.parameters()):
            assert torch.equal(pe, pg), (i, n)
        for ae, ag in zip(eager.optimizer.accum, graphed.optimizer.accum):
            assert torch.equal(ae, ag), i
    assert graphed.replays == steps - 2, graphed.replays
    assert graphed.captures == 1 + len(graphed._B) and len(graphed._B) == 8
    # structural: no capture holds a memset node (their order against the
    # kernels is not kept under the runtime's default graph packet capture)
    assert len(graphed.census) == 9
    assert all(c.get("memset", 0) == 0 and c.get("kernel", 0) > 100
               for c in graphed.census.values()), graphed.census
    from detectron2_tensorflow_amd import _C
    _C.raise_on_errors(dev)
    print("mask rows per step", rows, "node census", graphed.census)
    return graphed, rows


def test_graphed_trainer_matches_eager_trainer(dev, monkeypatch):
    _alternating_steps(dev, monkeypatch, 256, 320, 7, 4, (11, 12))


def test_graphed_trainer_matches_eager_trainer_1333x800(dev, monkeypatch):
    """The geometry bench.py times: the K = 256 stream
    1x1, the large-grid warp-specialised conv plans and the 8 B[R] graphs at
    the bench's shapes, replayed over batches with different foreground
    counts, equal to Trainer.step bit for bit."""
    # 48 GT per image in the first batch (each appended GT box is a foreground
    # proposal: >= 96 mask rows), 2 in the second
    graphed, rows = _alternating_steps(dev, monkeypatch, 800, 1333, 5, 3, (1000, 1001), num_gt=48)
    assert len(set(rows[1:])) >= 2, rows  # the replays used more than one B[R]


def test_graphed_trainer_rejects_other_batch_shape(dev):
    from detectron2_tensorflow_amd.engine.graphed import GraphedTrainer
    from detectron2_tensorflow_amd.utils.synthetic import synthetic_train_batch
    cfg, model = _model(dev)
    tr = GraphedTrainer(cfg, model, warmup=1)
    b = synthetic_train_batch(2, 256, 320, 3, dev)
    tr.step(b)  # eager warm-up
    tr.step(b)  # capture + replay
    assert tr.replays == 1
    with pytest.raises(ValueError, match="captured for"):
        tr.step(synthetic_train_batch(2, 256, 384, 3, dev))
