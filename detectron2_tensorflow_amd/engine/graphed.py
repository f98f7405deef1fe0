"""The training step replayed from hipGraphs (lib/engine/trainer.py:116-199).

Status (r5): bit-identical to ``Trainer.step`` over steps that change the
batch and the mask-branch row count (tests/test_gpu_graphed.py).  Two causes
of the r4 failures were found and fixed:

* the replay FAULTS: host-filled launch tables (fold / optimizer pointer
  tables) were allocated inside the capture, from the graph pool, where a
  captured temporary could share their bytes and overwrite them at replay
  (utils/capture.py; tools/graph_audit.py proves it from the allocator trace:
  15 of 17 tables overlapped captured allocations, 0 with the fix);
* the replay DIVERGENCE once the batch changes: memset nodes are not ordered
  against the kernel nodes around them when the HIP runtime pre-records the
  graph's kernels as AQL packets (its graph "packet capture"): the matcher's
  zeroed per-GT best IoU (an atomic max) and torch's global-reduction
  semaphores (the box head's bias gradient) kept a previous replay's values
  (tools/graph_diff.py: eager-exact with DEBUG_CLR_GRAPH_PACKET_CAPTURE=0,
  divergent with it on).

r6 made the captures memset-free instead of turning the runtime's packet
capture off: the library fills with kernels (d2mi::fill_bytes), and the one
torch op that still issued a memset -- the reduction behind the box head's
fc2 / predictor bias gradients, whose cross-block semaphores torch zeroes
with hipMemsetAsync -- is the library's fixed-order column sum
(layers/wrappers.py: _LinearBiasFn).  Every capture is censused before it
is instantiated (d2mi_graph_census; ``census``): 0 memset nodes in A and in
every B[R] (tools/graph_nodes.py names any op that adds one), and a capture
that holds one is refused while packet capture is on.  With the runtime's
defaults the replays are bit-identical to the eager step at 256x320 and at
the bench's 1333x800 (tests/test_gpu_graphed.py), and the bench runs the
same with packet capture on or off (profiles/r6b_bench_pkt_*.json).

The eager ``Trainer.step`` enqueues ~550 launches per iteration from Python
(autograd engine, custom Functions, ctypes): on an MI355X that host work is
0.6-0.75 of the step's wall time, so one faster kernel away from binding the
step.  Here the same step is captured into hipGraphs once and replayed:

* graph A: the forward (backbone, FPN, RPN + its losses, ROI sampling, box
  branch + losses) up to the one value the host must read -- the number of
  foreground proposals, which sizes the compacted mask branch (the
  reference's ``select_foreground_proposals``, roi_heads.py:35-62);
* graph B[R], one per possible mask-branch row count R (a multiple of 32:
  8 graphs for 2 images x 128 foreground slots, all captured right after
  A): the mask branch forward + loss, the total loss, the whole backward (through graph A's retained autograd graph), the all-reduce
  (world size 1: none; see below) and the fused Momentum-SGD update with the LR read
  from the device (``d2mi_momentum_sgd_ex``).

A step is then: copy the batch into the captured input tensors (when the
caller passes others), write the LR, replay A, read the foreground count
(the step's one host synchronisation, as in the eager step), replay B[R].
The arithmetic is the eager step's: the same kernels with the same arguments in the same order, so the updated
weights are bit-identical to ``Trainer.step`` on the same inputs (tests).

Every B graph shares graph A's memory pool: A's outputs and saved tensors
stay alive (the retained autograd graph and the deferred mask loss hold
them), and the B graphs, never replayed concurrently, reuse each other's
freed temporaries.  The caches keyed on parameter versions (folded /
packed weights) are made stale before A is captured, so A re-folds and
re-packs every trainable layer at each replay; nothing bumps a version while
the graphs are in use, and an eager step (``eager_step``) marks them stale
again first.

Data parallel (r6): with the bucketed all-reduce active (world > 1) B[R]
ends after the backward and its bucket copies; the host launches the
buckets' all-reduces right after launching B[R] (engine/reducer.py, capture
form), and a last graph U (the update over the reduced buckets) replays
after them.
"""
import os

import torch

from ..layers import convolutional
from ..modeling.roi_heads.roi_heads import DeferredMaskLoss, StandardROIHeads
from ..utils import capture, host_sync
from .trainer import Trainer


NODE_KINDS = ("kernel", "memcpy", "memset", "host", "graph", "empty", "wait_event",
              "event_record", "ext_signal", "ext_wait", "mem_alloc", "mem_free",
              "memcpy_from_symbol", "memcpy_to_symbol", "batch_mem_op")


def _census_dict(counts):
    return {NODE_KINDS[i]: int(c) for i, c in enumerate(counts) if c}


def graph_census(g):
    """{node kind: count} of a captured ``torch.cuda.CUDAGraph(keep_graph=True)``
    that is not instantiated yet (d2mi_graph_census)."""
    import ctypes
    from .. import _C
    counts = (ctypes.c_longlong * len(NODE_KINDS))()
    _C.check(_C.lib().d2mi_graph_census(ctypes.c_void_p(g.raw_cuda_graph()), counts,
                                        len(NODE_KINDS)), "d2mi_graph_census")
    return _census_dict(counts)


def capture_census(device=None):
    """The same census of the graph the current stream is capturing into
    (None when it is not capturing; d2mi_capture_census)."""
    import ctypes
    from .. import _C
    counts = (ctypes.c_longlong * len(NODE_KINDS))()
    rc = _C.lib().d2mi_capture_census(_C.stream_of(device), counts, len(NODE_KINDS))
    _C.check(min(rc, 0), "d2mi_capture_census")
    return None if rc == 1 else _census_dict(counts)


def packet_capture_on():
    """Whether the HIP runtime pre-records captured kernels as AQL packets
    (its default; DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 read at runtime start
    turns it off)."""
    return os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "1") not in ("0", "false", "False")


def _flatten(tree, prefix=()):
    """(path, tensor) leaves of a nested dict of tensors, in key order."""
    out = []
    for k in sorted(tree):
        v = tree[k]
        if isinstance(v, dict):
            out += _flatten(v, prefix + (k,))
        elif torch.is_tensor(v):
            out.append((prefix + (k,), v))
    return out


def _clone_tree(tree):
    return {k: (_clone_tree(v) if isinstance(v, dict) else
                v.clone() if torch.is_tensor(v) else v) for k, v in tree.items()}


class GraphedTrainer(Trainer):
    """``Trainer`` whose steps replay captured hipGraphs (see the module
    docstring).  ``warmup``: eager steps before the capture (at least one:
    allocator, workspaces, per-shape caches).  Falls back to the eager step when the
    process group has more than one rank."""

    def __init__(self, cfg, model, warmup=1, experimental=False, wgrad_side=False, **kwargs):
        """experimental: accepted for the r4 call sites (no longer needed)."""
        super().__init__(cfg, model, **kwargs)
        # >= 1: the first eager step makes the per-shape caches, workspaces and
        # the optimizer / fold tables, none of which may be created in a capture
        self.warmup = max(1, int(warmup))
        self.heads = [m for m in model.modules() if isinstance(m, StandardROIHeads)]
        # any world size (r6): the collectives stay outside the graphs.
        # Capturing the bucketed all-reduce itself fails over RCCL (the
        # process group's watchdog queries the events of collectives recorded
        # inside a capture) and gloo cannot be captured at all, so with the
        # reducer active B[R] ends after the backward's bucket copies, the
        # host launches the all-reduces after it (engine/reducer.py, capture
        # form), and one more graph, U, holds the update.
        self.enabled = next(model.parameters()).is_cuda
        self._U = None
        # r6: capture the backward with every conv's weight gradient on a side
        # stream (layers/convolutional.py WGRAD_STREAM).  Off by default:
        # bit-identical, but no faster -- 105.3 / 105.8 vs 105.6 / 106.1 img/s
        # in alternating bench runs (profiles/r6l_bench_wgrad_side_ab.txt): the
        # warp-specialised convs hold a whole CU each, so the branches contend
        self.wgrad_side = bool(wgrad_side)
        self._wgrad_stream = None
        self._eager = 0
        self._pool = None
        self._A = None
        self._B = {}
        self._static = None
        self._leaves = None
        self._losses = None
        self._deferred = None
        self._lr_dev = None
        self._stream = None
        self.captures = 0
        self.replays = 0
        # node kinds of every capture ("A", "B<rows>" -> {kind: count}),
        # checked before the graph is instantiated (_finish)
        self.census = {}
        # a directory: every captured graph is written there as a DOT file
        # (hipGraphDebugDotPrint; tools/graph_dump.py) -- a diagnosis that
        # replays nothing
        self.debug_dump_dir = None

    # ------------------------------------------------------------------ state
    def _mark_stale(self):
        """Make every version-keyed cache of a trainable layer (FrozenBN folds,
        packed weights, the RPN head's fused 1x1 weights) miss once."""
        torch.autograd.graph.increment_version(self.optimizer.params)

    def _on_stream(self, fn, *args):
        """fn(*args) on the trainer's own stream -- the eager warm-up steps, the
        captures and the replays alike, so every autograd node (AccumulateGrad
        included) lives on the stream the graphs are captured on -- ordered
        after the caller's stream on entry and before it on exit."""
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=next(self.model.parameters()).device)
        caller = torch.cuda.current_stream(self._stream.device)
        self._stream.wait_stream(caller)
        with torch.cuda.stream(self._stream):
            out = fn(*args)
        caller.wait_stream(self._stream)
        return out

    def eager_step(self, batched_inputs):
        """One eager ``Trainer.step`` (e.g. with kernel timers on).  It reads
        the current weights: the caches are marked stale before it, and it
        leaves no state the graphs depend on."""
        if not self.enabled:
            return Trainer.step(self, batched_inputs)
        if self._A is not None:
            self._mark_stale()
        for h in self.heads:
            h.defer_mask_loss = False
        return self._on_stream(Trainer.step, self, batched_inputs)

    def _load(self, batched_inputs):
        leaves = _flatten(batched_inputs)
        if [p for p, _ in leaves] != [p for p, _ in self._leaves]:
            raise ValueError("graphed step: the batch has other fields than the captured one")
        for (path, v), (_, s) in zip(leaves, self._leaves):
            if v.shape != s.shape or v.dtype != s.dtype:
                raise ValueError(f"graphed step: {'/'.join(path)} is {tuple(v.shape)} "
                                 f"{v.dtype}, the graphs were captured for {tuple(s.shape)} "
                                 f"{s.dtype}")
            if v.data_ptr() != s.data_ptr():
                s.copy_(v, non_blocking=True)

    # ---------------------------------------------------------------- capture
    def _new_graph(self):
        # keep_graph: the captured hipGraph stays readable until _finish has
        # taken its node census and instantiated it
        g = torch.cuda.CUDAGraph(keep_graph=True)
        if self.debug_dump_dir:
            g.enable_debug_mode()
        return g

    def _finish(self, g, name):
        """Census the capture's nodes, refuse memset nodes while the HIP
        runtime's graph packet capture is on, instantiate."""
        census = graph_census(g)
        self.census[name] = census
        if census.get("memset", 0) and packet_capture_on():
            raise RuntimeError(
                f"graphed step: capture {name} holds {census['memset']} memset node(s) and the "
                "HIP runtime's graph packet capture is on (DEBUG_CLR_GRAPH_PACKET_CAPTURE is "
                "not 0): their order against the kernels around them is not kept, and replays "
                "diverge from the eager step (r5).  tools/graph_nodes.py names the ops that "
                "issue them")
        g.instantiate()

    def _dump(self, g, name):
        if self.debug_dump_dir:
            import os
            os.makedirs(self.debug_dump_dir, exist_ok=True)
            g.debug_dump(os.path.join(self.debug_dump_dir, f"graph_{name}.dot"))

    def _capture_forward(self, batched_inputs):
        self._static = _clone_tree(batched_inputs)
        self._leaves = _flatten(self._static)
        dev = self._leaves[0][1].device
        self._lr_dev = torch.zeros((), dtype=torch.float32, device=dev)
        for h in self.heads:
            h.defer_mask_loss = True
        if not self.model.training:
            self.model.train()
        self.optimizer.zero_grad()
        self.reducer.reset()
        self._mark_stale()
        torch.cuda.synchronize(dev)
        self._pool = torch.cuda.graph_pool_handle()
        g = self._new_graph()
        # r5: graph A ends with the foreground count's copy into pinned host
        # memory, so the host's one read is a wait on the replay alone (before:
        # wait for A, then enqueue a device-to-host copy and wait for it -- the
        # copy started ~60-140 us after A's last kernel, the device idle)
        self._count_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        capture.begin(dev)  # (outside the capture: see utils/capture.py)
        with torch.cuda.graph(g, pool=self._pool, stream=self._stream,
                              capture_error_mode="thread_local"):
            losses = self.model(self._static)
            for v in losses.values():
                if isinstance(v, DeferredMaskLoss):
                    self._count_host.copy_(v.count.reshape(1).to(torch.int64), non_blocking=True)
        self._dump(g, "A")
        self._finish(g, "A")
        self._keep = []
        capture.flush(self._keep)
        deferred = [v for v in losses.values() if isinstance(v, DeferredMaskLoss)]
        if len(deferred) > 1:
            raise RuntimeError("graphed step: more than one deferred mask loss")
        self._A = g
        self._losses = losses
        self._deferred = deferred[0] if deferred else None
        self.captures += 1
        # every B graph now, while the layers' cached packed weights are the
        # ones graph A refreshes (a later eager step re-points those caches)
        d = self._deferred
        for rows in (sorted({d.rows_for(n) for n in range(d.slots + 1)}) if d else [None]):
            self._capture_rest(rows)

    def _capture_rest(self, rows):
        """Graph B[rows]: mask branch, total loss, backward, update."""
        self.optimizer.zero_grad()
        keep = []
        g = self._new_graph()
        dev = self._lr_dev.device
        # the loss values land in a buffer of the ordinary pool: no later
        # capture's temporary (the shared pool) can overwrite them before the
        # host reads them
        nvals = len(self._losses) + 1
        vals = torch.empty(nvals, dtype=torch.float32, device=dev)
        capture.begin(dev)
        with torch.cuda.graph(g, pool=self._pool, stream=self._stream,
                              capture_error_mode="thread_local"):
            out = {k: (v.compute(rows) if isinstance(v, DeferredMaskLoss) else v)
                   for k, v in self._losses.items()}
            total = torch.stack(self._loss_terms(out)).sum()
            seed = self._seed
            if seed is None or seed.device != total.device or seed.dtype != total.dtype:
                seed = self._seed = torch.ones_like(total)
            # retain graph A's autograd graph: a later row count is captured
            # by another backward through it
            dp = self.reducer.active
            if dp:
                self.reducer.begin_capture()
            # the convs' weight gradients on a side stream beside their data
            # gradients: forked branches of the captured graph (r6)
            if self.wgrad_side:
                if self._wgrad_stream is None:
                    self._wgrad_stream = torch.cuda.Stream(device=dev)
                convolutional.WGRAD_STREAM["stream"] = self._wgrad_stream
            try:
                total.backward(seed, retain_graph=True)
            finally:
                convolutional.WGRAD_STREAM.pop("stream", None)
            self.reducer.finish()
            events = self.reducer.end_capture() if dp else None
            if not dp:
                self.optimizer.step_captured(self._lr_dev)
            vals.copy_(torch.stack([t.detach() for t in self._loss_terms(out)] + [total.detach()]))
        capture.flush(keep)
        values = vals
        self._dump(g, f"B{rows}")
        self._finish(g, f"B{rows}")
        if dp and self._U is None:
            self._capture_update(dev)
        self.optimizer.zero_grad()
        keys = list(out) + ["total_loss"]
        self._B[rows] = (g, values, keys, keep, events)
        self.captures += 1

    def _capture_update(self, dev):
        """Graph U (reducer active): the fused Momentum-SGD update over the
        gradients as views of the all-reduced buckets -- the same pointers
        after every B[R], so one graph serves them all."""
        keep = []
        g = self._new_graph()
        capture.begin(dev)
        with torch.cuda.graph(g, pool=self._pool, stream=self._stream,
                              capture_error_mode="thread_local"):
            self.optimizer.step_captured(self._lr_dev)
        capture.flush(keep)
        self._dump(g, "U")
        self._finish(g, "U")
        self._U = (g, keep)
        self.captures += 1

    # ------------------------------------------------------------------- step
    def step(self, batched_inputs):
        if not self.enabled:
            return Trainer.step(self, batched_inputs)
        if self._A is None and self._eager < self.warmup:
            self._eager += 1
            return self.eager_step(batched_inputs)
        return self._on_stream(self._graph_step, batched_inputs)

    def _graph_step(self, batched_inputs):
        if self._A is None:
            try:
                self._capture_forward(batched_inputs)
            except BaseException:
                capture.discard()
                raise
        self._load(batched_inputs)
        self._lr_dev.fill_(float(self.lr(self.iter)))
        if self._deferred is not None:
            host_sync.arm_pinned(self._count_host)
        self._A.replay()
        rows = None
        if self._deferred is not None:
            nfg = host_sync.read_pinned(self._count_host)[0]  # the step's one host read
            rows = self._deferred.rows_for(nfg)
            for h in self.heads:
                h.last_mask_rows = rows
        g, values, keys, _, events = self._B[rows]
        g.replay()
        if events is not None:
            # the buckets' all-reduces after the replayed backward, then the
            # update after the last
            self.reducer.launch_captured(events)
            self.reducer.wait_captured()
            self._U[0].replay()
        self.replays += 1
        self.iter += 1
        # (a copy: the next replay rewrites ``values``)
        values = values.clone()
        return {k: values[i] for i, k in enumerate(keys)}
