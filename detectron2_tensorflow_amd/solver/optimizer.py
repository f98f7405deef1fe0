"""Momentum SGD with the reference's regulariser and gradient clipping.

trainer.py:116-139 builds: total loss = mean of clone losses + L2 regularisers
(regularizer.py:6-24: slim.l2_regularizer(scale) = scale * sum(w^2) / 2 per
variable, with WEIGHT_DECAY for "weights", WEIGHT_DECAY_BIAS for "bias",
WEIGHT_DECAY_NORM for "gamma"/"beta"; a zero scale adds nothing), then
slim.learning.clip_gradient_norms — clip_by_norm of EACH gradient tensor
separately to CLIP_GRADIENTS_BY_NORM — then tf.train.MomentumOptimizer
(accum = m * accum + g; var -= lr * accum).

Here the regulariser enters as its gradient (scale * w) and every step is a
handful of multi-tensor (torch._foreach_*) launches over all parameters: no
per-parameter Python loop on the hot path and no host synchronisation.
"""
import torch


def param_groups(model, cfg):
    """Trainable parameters grouped by regulariser scale (regularizer.py:12-22)."""
    s = cfg.SOLVER
    groups = {}
    for name, p in model.named_parameters():
        if not p.requires_grad:
            continue
        leaf = name.rsplit(".", 1)[-1]
        if leaf in ("gamma", "beta"):
            wd = s.WEIGHT_DECAY_NORM
        elif leaf == "bias":
            wd = s.WEIGHT_DECAY_BIAS
        else:
            wd = s.WEIGHT_DECAY
        groups.setdefault(float(wd), []).append(p)
    return [{"params": v, "weight_decay": k} for k, v in sorted(groups.items())]


class MomentumSGD:
    def __init__(self, groups, momentum=0.9, clip_norm=10.0):
        self.groups = groups
        self.momentum = float(momentum)
        self.clip_norm = float(clip_norm)
        self.params = [p for g in groups for p in g["params"]]
        self.accum = [torch.zeros_like(p) for p in self.params]

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    @torch.no_grad()
    def step(self, lr):
        grads = []
        for g in self.groups:
            ps = g["params"]
            gs = [p.grad if p.grad is not None else torch.zeros_like(p) for p in ps]
            if g["weight_decay"] > 0:
                gs = torch._foreach_add(gs, ps, alpha=g["weight_decay"])
            grads.extend(gs)
        if self.clip_norm > 0:
            norms = torch.stack(torch._foreach_norm(grads))
            # clip_by_norm: g * clip / max(|g|, clip)
            scale = self.clip_norm / torch.clamp(norms, min=self.clip_norm)
            torch._foreach_mul_(grads, list(scale.unbind()))
        torch._foreach_mul_(self.accum, self.momentum)
        torch._foreach_add_(self.accum, grads)
        torch._foreach_add_(self.params, self.accum, alpha=-float(lr))
