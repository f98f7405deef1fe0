"""Data-parallel training step (lib/engine/trainer.py:43-199, model_deploy.py:122-438).

One process per GPU.  Each rank runs the model on its own shard of the global
batch (fixing the reference's shared-batch quirk, trainer.py:63 — SURVEY.md
section 8a), backward overlaps the bucketed RCCL gradient all-reduce
(engine/reducer.py), and every rank applies the identical Momentum-SGD update
(solver/optimizer.py) with the host-side LR schedule (solver/learning_rate.py).

A step enqueues work only: the losses come back as device tensors and the
caller decides when to synchronise (bench.py brackets K steps with one
barrier + synchronize on each side).
"""
import torch
import torch.distributed as dist

from ..solver import MomentumSGD, build_learning_rate, param_groups
from .reducer import BucketedAllReduce


def get_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def broadcast_parameters(model, src=0, group=None):
    """Start every replica from rank src's weights (slim's single variable copy)."""
    if get_world()[0] == 1:
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src, group=group)


class Trainer:
    def __init__(self, cfg, model, bucket_bytes=32 << 20, group=None, start_step=0,
                 reducer_always=False):
        """reducer_always: run the bucketed all-reduce (hooks + collectives)
        at world size 1 too -- the RCCL code path on one GPU (tests)."""
        self.cfg = cfg
        self.model = model
        self.world, self.rank = get_world()
        broadcast_parameters(model, group=group)
        self.optimizer = MomentumSGD(param_groups(model, cfg), momentum=cfg.SOLVER.MOMENTUM,
                                     clip_norm=cfg.SOLVER.CLIP_GRADIENTS_BY_NORM)
        self.reducer = BucketedAllReduce(self.optimizer.params, bucket_bytes, group,
                                         always=reducer_always)
        self.lr = build_learning_rate(cfg)
        self.iter = start_step
        self._seed = None

    @staticmethod
    def _loss_terms(losses):
        """Every loss as a 0-d float32 tensor on one device (what the stack
        needs).  A Python number becomes a constant tensor; a tensor of
        another float dtype is cast (no launch when it already is f32); a
        non-scalar or integer loss raises, naming its key."""
        terms, dev = [], None
        for k, v in losses.items():
            if torch.is_tensor(v):
                if v.numel() != 1 or not (v.is_floating_point()):
                    raise TypeError(f"loss {k!r} must be a scalar float tensor, got "
                                    f"{v.dtype} of shape {tuple(v.shape)}")
                dev = dev or v.device
                if v.device != dev:
                    raise ValueError(f"loss {k!r} is on {v.device}, the others on {dev}")
                terms.append(v.reshape(()) if v.dtype == torch.float32
                             else v.reshape(()).to(torch.float32))
            elif isinstance(v, (int, float)):
                terms.append(float(v))
            else:
                raise TypeError(f"loss {k!r} has unsupported type {type(v).__name__}")
        if dev is None:
            raise ValueError("no tensor loss to differentiate")
        return [t if torch.is_tensor(t) else torch.tensor(t, dtype=torch.float32, device=dev)
                for t in terms]

    def step(self, batched_inputs):
        """One iteration: forward + losses, backward with the overlapped
        all-reduce, clip + momentum update.  Returns the loss dict (device)."""
        if not self.model.training:  # (train() walks every module: host time per step)
            self.model.train()
        self.optimizer.zero_grad()
        self.reducer.reset()
        losses = self.model(batched_inputs)
        # one stack + one sum (not a chain of adds: 2 launches, and the
        # backward hands every loss the same seed without a kernel)
        total = torch.stack(self._loss_terms(losses)).sum()
        # the backward seed: one cached 1.0 per device (not a fill per step)
        seed = self._seed
        if seed is None or seed.device != total.device or seed.dtype != total.dtype:
            seed = self._seed = torch.ones_like(total)
        total.backward(seed)
        self.reducer.finish()
        self.optimizer.step(self.lr(self.iter))
        self.iter += 1
        # detached: a returned loss must not keep this step's autograd graph
        # (and its AccumulateGrad nodes, bound to this step's stream) alive
        losses = {k: (v.detach() if torch.is_tensor(v) else v) for k, v in losses.items()}
        losses["total_loss"] = total.detach()
        return losses
