"""The RCCL code path of engine/reducer.py on ONE GPU (tests/test_gpu_dp.py).

A child process (never an exec of the test process) initialises
torch.distributed with the "nccl" backend (RCCL on ROCm) at world size 1 on
cuda:0 and trains Mask R-CNN R50-FPN at 256x320 for 3 Trainer.steps with the
bucketed all-reduce FORCED on (Trainer(reducer_always=True): the
post-accumulate-grad hooks, the flat buckets, one RCCL all-reduce per bucket
on the communicator's stream, finish()'s waits and .grad views), the second
step with the per-bucket timing events.  It then replays the same 3 steps
on a second model built from the same seed without the reducer, and (r6) on
a third with GraphedTrainer and the RCCL reducer (graph replays, the
all-reduces launched on the replay's bucket events).  An
all-reduce of one rank is exact (x * 1.0, summed once), so the two parameter
vectors must be bit-identical.  Writes <outdir>/rccl.pt.

    python tests/rccl_worker.py <outdir>      (MASTER_ADDR / MASTER_PORT in env)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dp_worker import CATS, batch_of, build, flat  # noqa: E402

STEPS = 3


def main(out):
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    from detectron2_tensorflow_amd.engine import Trainer
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    _C.load()
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, "configs", "COCO-InstanceSegmentation",
                                     "mask_rcnn_R_50_FPN_1x.yaml"))
    cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT = "raw"
    cfg.SOLVER.WARMUP_ITERS = 0
    finalize(cfg, True, 1, CATS)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    backend = dist.get_backend()
    calib = batch_of(0, dev)
    batch = batch_of(0, dev)
    res = {"backend": backend}
    from detectron2_tensorflow_amd.engine.graphed import GraphedTrainer
    for arm in ("rccl", "plain", "rccl_graphed"):
        model = build(cfg, dev, calib)
        if arm == "rccl_graphed":
            # r6: the graphed step with the RCCL reducer: B[R] records the
            # buckets' ready events, the host launches the all-reduces on them,
            # the update graph U replays after (engine/graphed.py)
            trainer = GraphedTrainer(cfg, model, warmup=1, bucket_bytes=8 << 20,
                                     reducer_always=True)
        else:
            trainer = Trainer(cfg, model, bucket_bytes=8 << 20, reducer_always=(arm == "rccl"))
        assert trainer.reducer.active == (arm != "plain")
        for s in range(STEPS):
            torch.cuda.manual_seed(1000 * s)
            trainer.reducer.timing = arm == "rccl" and s == STEPS - 1
            losses = trainer.step(batch)
        torch.cuda.synchronize()
        res[arm] = flat(model)
        res[arm + "_losses"] = {k: float(v) for k, v in losses.items()}
        if arm == "rccl":
            res["timeline"] = trainer.reducer.timeline()
            res["buckets"] = len(trainer.reducer.buckets)
        if arm == "rccl_graphed":
            res["replays"] = trainer.replays
            res["census"] = trainer.census
    _C.raise_on_errors(dev)
    dist.destroy_process_group()
    torch.save(res, os.path.join(out, "rccl.pt"))


if __name__ == "__main__":
    main(sys.argv[1])
