"""Momentum SGD with the reference's regulariser and gradient clipping.

trainer.py:116-139 builds: total loss = mean of clone losses + L2 regularisers
(regularizer.py:6-24: slim.l2_regularizer(scale) = scale * sum(w^2) / 2 per
variable, with WEIGHT_DECAY for "weights", WEIGHT_DECAY_BIAS for "bias",
WEIGHT_DECAY_NORM for "gamma"/"beta"; a zero scale adds nothing), then
slim.learning.clip_gradient_norms — clip_by_norm of EACH gradient tensor
separately to CLIP_GRADIENTS_BY_NORM — then tf.train.MomentumOptimizer
(accum = m * accum + g; var -= lr * accum).

Here the regulariser enters as its gradient (scale * w).  On the GPU the
whole update is d2mi_momentum_sgd: two launches over a table of every
trainable tensor (per-tensor norms as fixed-order chunk sums, then clip +
momentum + update fused), no host synchronisation; the per-step part of the
table (the gradient pointers) goes up through a small ring of pinned host
buffers.  Off the GPU (the gloo / CPU tests) the same arithmetic runs as
torch._foreach_* ops.
"""
import numpy as np
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

    _TENSOR_DT = np.dtype([("w", "<u8"), ("g", "<u8"), ("accum", "<u8"), ("numel", "<i8"),
                           ("wd", "<f4"), ("first_chunk", "<i4"), ("num_chunks", "<i4"),
                           ("pad", "<i4")])
    _CHUNK_DT = np.dtype([("tensor", "<i4"), ("pad", "<i4"), ("begin", "<i8"), ("end", "<i8")])
    _RING = 4

    def _fused_init(self):
        from .. import _C
        lib = _C.load()
        tb, cb, per = (_C.ctypes.c_int(), _C.ctypes.c_int(), _C.ctypes.c_int())
        lib.d2mi_sgd_table_sizes(_C.ctypes.byref(tb), _C.ctypes.byref(cb), _C.ctypes.byref(per))
        if tb.value != self._TENSOR_DT.itemsize or cb.value != self._CHUNK_DT.itemsize:
            raise RuntimeError("d2mi_momentum_sgd table layout mismatch")
        dev = self.params[0].device
        wd = [g["weight_decay"] for g in self.groups for _ in g["params"]]
        tab = np.zeros(len(self.params), self._TENSOR_DT)
        chunks = []
        for i, (p, a) in enumerate(zip(self.params, self.accum)):
            if not (p.is_contiguous() and a.is_contiguous() and p.dtype == torch.float32):
                raise RuntimeError("fused Momentum-SGD needs contiguous f32 parameters")
            n = p.numel()
            tab[i] = (p.data_ptr(), 0, a.data_ptr(), n, wd[i], len(chunks),
                      max(1, -(-n // per.value)), 0)
            for b in range(0, max(n, 1), per.value):
                chunks.append((i, 0, b, min(n, b + per.value)))
        ctab = np.array(chunks, self._CHUNK_DT)
        self._tab = tab
        self._nchunks = len(chunks)
        self._chunks_dev = torch.from_numpy(ctab.view(np.uint8).copy()).to(dev)
        self._tab_dev = torch.empty(tab.nbytes, dtype=torch.uint8, device=dev)
        self._partial = torch.empty(self._nchunks, dtype=torch.float32, device=dev)
        self._ring = [torch.empty(tab.nbytes, dtype=torch.uint8).pin_memory()
                      for _ in range(self._RING)]
        self._ring_ev = [None] * self._RING
        self._ring_i = 0
        self._lib = lib

    def _step_fused(self, lr):
        from .. import _C
        if getattr(self, "_tab", None) is None:
            self._fused_init()
        grads = []
        for i, p in enumerate(self.params):
            g = p.grad
            if g is not None and not g.is_contiguous():
                g = g.contiguous()  # freed after the launch: stream-ordered reuse only
            grads.append(g)
            self._tab["g"][i] = 0 if g is None else g.data_ptr()
        k = self._ring_i
        self._ring_i = (k + 1) % self._RING
        if self._ring_ev[k] is not None:  # the slot's previous upload has left
            self._ring_ev[k].synchronize()
        self._ring[k].numpy()[:] = self._tab.view(np.uint8)
        stream = torch.cuda.current_stream(self._tab_dev.device)
        self._tab_dev.copy_(self._ring[k], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        self._ring_ev[k] = ev
        rc = self._lib.d2mi_momentum_sgd(_C.ptr(self._tab_dev), _C.ptr(self._chunks_dev),
                                         self._nchunks, _C.ptr(self._partial),
                                         float(self.clip_norm), float(self.momentum), float(lr),
                                         _C.stream_of(self._tab_dev.device))
        _C.check(rc, "d2mi_momentum_sgd")
        # the kernel wrote the parameters through raw pointers: bump their
        # version counters as an in-place torch op would (the packed-weight
        # and fused-head caches key on them)
        torch.autograd.graph.increment_version(self.params)

    def step_captured(self, lr_dev):
        """The fused update for a training step being captured into a hipGraph
        (engine/graphed.py).  The table of this capture's gradient pointers is
        constant across replays: the captured launches read it from a device
        buffer of their own that utils.capture fills after the capture (no
        host memory or copy node inside the graph).  The learning rate is read
        from the device float ``lr_dev`` at run time (d2mi_momentum_sgd_ex).
        No version bump: nothing runs at capture time, and the packed-weight
        caches must keep the keys the captured forward was recorded with."""
        from .. import _C
        from ..utils import capture
        if getattr(self, "_tab", None) is None:
            self._fused_init()
        tab = self._tab.copy()
        for i, p in enumerate(self.params):
            g = p.grad
            if g is not None and not g.is_contiguous():
                raise RuntimeError("captured Momentum-SGD needs contiguous gradients")
            tab["g"][i] = 0 if g is None else g.data_ptr()
        dev_tab = capture.table(tab, self._tab_dev.device, "momentum-sgd")
        rc = self._lib.d2mi_momentum_sgd_ex(_C.ptr(dev_tab), _C.ptr(self._chunks_dev), self._nchunks,
                                            _C.ptr(self._partial), float(self.clip_norm),
                                            float(self.momentum), 0.0, _C.ptr(lr_dev),
                                            _C.stream_of(dev_tab.device))
        _C.check(rc, "d2mi_momentum_sgd_ex")

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    @torch.no_grad()
    def step(self, lr):
        if self.params and self.params[0].is_cuda:
            return self._step_fused(lr)
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
