"""One rank of the real-model data-parallel test (tests/test_gpu_dp.py).

Launched by the test as a child process per rank (never an exec of the test
process), every rank on cuda:0, torch.distributed over gloo (the collective
code path of engine/reducer.py is backend-agnostic; RCCL is the driver's
8-GPU run).  Each rank builds Mask R-CNN R50-FPN at 256x320 from the same
seed, trains 2 Trainer.steps on ITS OWN batch (rank 1's images carry fewer
GT boxes, so its ROI heads see fewer foreground rows and its mask branch a
different row count), and saves its flat parameter vector and losses after
each step.  Rank 0 then rebuilds the model and replays the two steps in one
process: per step the gradients of both batches (same RNG seeds as the
ranks used), averaged as the reducer does (g * 1/world, summed), one
Momentum-SGD update -- model_deploy.py:203-205's mean of the per-clone
losses -- and saves those parameter vectors too.

    python tests/dp_worker.py <outdir> [eager|graphed]   (RANK / WORLD_SIZE / MASTER_* in env)

"graphed" (r6): each rank also trains a second replica of the same model
with engine/graphed.py's GraphedTrainer on the same batches, right after the
eager step -- step 0 its eager warm-up, then graph A + B[R] + the update
graph U replayed, the bucketed all-reduces launched between B[R] and U
(engine/reducer.py, capture form) -- for 3 steps.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CATS = {"num_thing_classes": 80, "num_stuff_classes": 53, "stuff_ignore_value": 0}
STEPS = {"eager": 2, "graphed": 3}


def build(cfg, dev, calib_batch):
    from detectron2_tensorflow_amd.modeling import build_model
    from detectron2_tensorflow_amd.utils.synthetic import calibrate_rcnn_scores
    torch.manual_seed(0)
    model = build_model(cfg).to(dev).train()
    calibrate_rcnn_scores(model, calib_batch)
    model.train()
    return model


def batch_of(rank, dev):
    from detectron2_tensorflow_amd.utils.synthetic import synthetic_train_batch
    # rank 1: 2 GT boxes per image instead of 7 (fewer foreground ROIs)
    return synthetic_train_batch(2, 256, 320, 100 + rank, dev, num_gt=7 if rank == 0 else 2)


def seed(step, rank):
    return 1000 * step + rank


def flat(model):
    return torch.cat([p.detach().reshape(-1) for p in model.parameters() if p.requires_grad]).cpu()


def main(out, arm="eager"):
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    from detectron2_tensorflow_amd.engine import Trainer
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    _C.load()
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, "configs", "COCO-InstanceSegmentation",
                                     "mask_rcnn_R_50_FPN_1x.yaml"))
    cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT = "raw"
    cfg.SOLVER.WARMUP_ITERS = 0
    finalize(cfg, True, world, CATS)
    torch.backends.cudnn.deterministic = True
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calib = batch_of(0, dev)
    model = build(cfg, dev, calib)
    steps = STEPS[arm]
    trainer = Trainer(cfg, model)  # broadcasts rank 0's weights
    if arm == "graphed":
        # a second replica of the same model, trained by GraphedTrainer on the
        # same batches right after the eager one each step: bit-identical to it
        from detectron2_tensorflow_amd.engine.graphed import GraphedTrainer
        model_g = build(cfg, dev, calib)
        graphed = GraphedTrainer(cfg, model_g, warmup=1)
        assert graphed.enabled and graphed.reducer.active
    mine = batch_of(rank, dev)
    for s in range(steps):
        torch.cuda.manual_seed(seed(s, rank))
        losses = trainer.step(mine)
        rows = getattr(model.roi_heads, "last_mask_rows", None)
        rec = {"params": flat(model), "losses": {k: float(v) for k, v in losses.items()},
               "mask_rows": rows}
        if arm == "graphed":
            torch.cuda.manual_seed(seed(s, rank))
            lg = graphed.step(mine)
            rec.update(graphed_params=flat(model_g),
                       graphed_losses={k: float(v) for k, v in lg.items()},
                       graphed_rows=model_g.roi_heads.last_mask_rows,
                       replays=graphed.replays, census=graphed.census)
        torch.save(rec, os.path.join(out, f"rank{rank}_step{s}.pt"))
    _C.raise_on_errors(dev)
    dist.barrier()
    dist.destroy_process_group()
    if rank != 0:
        return
    # single-process replay with the averaged gradients
    from detectron2_tensorflow_amd.solver import MomentumSGD, build_learning_rate, param_groups
    ref = build(cfg, dev, calib)
    opt = MomentumSGD(param_groups(ref, cfg), momentum=cfg.SOLVER.MOMENTUM,
                      clip_norm=cfg.SOLVER.CLIP_GRADIENTS_BY_NORM)
    lr = build_learning_rate(cfg)
    batches = [batch_of(r, dev) for r in range(world)]
    for s in range(steps):
        acc = None
        for r, b in enumerate(batches):
            opt.zero_grad()
            torch.cuda.manual_seed(seed(s, r))
            sum(ref(b).values()).backward()
            g = [torch.zeros_like(p) if p.grad is None else p.grad.detach() * (1.0 / world)
                 for p in opt.params]
            acc = g if acc is None else [a + x for a, x in zip(acc, g)]
        for p, a in zip(opt.params, acc):
            p.grad = a
        opt.step(lr(s))
        torch.save({"params": flat(ref)}, os.path.join(out, f"single_step{s}.pt"))
    _C.raise_on_errors(dev)


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:3])
