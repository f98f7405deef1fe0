"""Bucketed gradient all-reduce overlapped with backward.

Replaces the reference's clone scheme (model_deploy.py:253-299, :408-438),
where every clone's gradients are summed with add_n on CPU:0 and the
variables travel host <-> device each step.  Here each rank holds its own
replica and its own shard of the batch; after backward the gradients of all
ranks are averaged with RCCL all-reduces (torch.distributed "nccl" backend)
so every replica applies the same update — the same arithmetic as the
reference's sum of per-clone losses x 1/num_clones.

Overlap: parameters are packed, in reverse registration order (the order
backward produces their gradients), into flat fp32 buckets of
``bucket_bytes``.  A post-accumulate-grad hook copies each gradient
(pre-scaled by 1/world) into its bucket slot; when every gradient of a bucket
has arrived the bucket's all-reduce is launched asynchronously on the
communicator's stream while backward continues.  Buckets are launched
strictly in index order on every rank (a bucket that completes early waits
for its predecessors), so the collective sequence is identical across ranks.
``finish()`` waits for the outstanding collectives and points each .grad at
its slice of the reduced bucket.

Bucket size: the ~44 M trainable fp32 gradients (~177 MB) of Mask R-CNN R50-FPN
split into 32 MB buckets give 6 collectives per step — large enough that each
ring all-reduce runs at xGMI link bandwidth, small enough that the first
launches early in backward.  The LAST bucket (the earliest-registered
parameters, whose gradients backward produces last) is capped at
``tail_bytes`` (4 MB, or bucket_bytes if smaller): its all-reduce is the one that cannot overlap the
backward, so it is kept short.

Timing (``timing = True``, bench.py's sampled step at world > 1): HIP events
record when each bucket became ready (on the compute stream, at its launch),
when its all-reduce completed (a side stream that waits only on that
collective), and the end of backward (the compute stream at ``finish()``);
``timeline()`` turns them into per-bucket ready / done times relative to the
end of backward, the all-reduce time the backward did NOT hide
(``exposed_ms``) and the collectives' busy time (reference semantics: the
clones' gradient sum of model_deploy.py:408-438 happens after the backward).

Graph-replayed steps (engine/graphed.py, r6).  A collective cannot sit
inside a captured hipGraph here (RCCL inside a capture trips the process
group's watchdog; gloo cannot be captured at all), so the reducer has a
capture form: while ``captured`` is set, the hooks' bucket copies are
captured with the backward but no collective is launched, and ``finish()``
only points the gradients at the buckets.  At replay the host launches the
backward graph, then every bucket's all-reduce in order on the side stream
after it (``launch_captured``), and ``wait_captured`` orders the update
graph after the last one.  The collectives therefore follow the replayed
backward instead of overlapping it (the eager hooks overlap them): an
external event-record node per bucket would restore the overlap, but torch
refuses external events on ROCm ("External events are disallowed in rocm").
"""
import torch
import torch.distributed as dist


class _Bucket:
    __slots__ = ("params", "offsets", "numel", "flat", "pending", "work")

    def __init__(self):
        self.params, self.offsets, self.numel = [], [], 0
        self.flat, self.pending, self.work = None, 0, None


class BucketedAllReduce:
    def __init__(self, params, bucket_bytes=32 << 20, group=None, tail_bytes=None, always=False):
        """always: arm the hooks and collectives at world size 1 too (the
        RCCL path exercised on one GPU: an all-reduce of one rank is exact)."""
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.active = self.world > 1 or (always and dist.is_initialized())
        self.timing = False
        # capture form (engine/graphed.py): ready buckets record events
        self.captured = False
        self._events = None
        self._tl = None
        self.params = [p for p in params if p.requires_grad]
        # partition in registration order starting from the tail bucket (at
        # most tail_bytes), then launch order = reverse registration order
        if tail_bytes is None:
            tail_bytes = min(4 << 20, bucket_bytes)
        groups, cur, cap, nbytes = [], [], tail_bytes, 0
        for p in self.params:
            if cur and nbytes + p.numel() * 4 > cap:
                groups.append(cur)
                cur, cap, nbytes = [], bucket_bytes, 0
            cur.append(p)
            nbytes += p.numel() * 4
        if cur:
            groups.append(cur)
        self.buckets = []
        self.where = {}
        for g in reversed(groups):
            b = _Bucket()
            for p in reversed(g):
                self.where[p] = (len(self.buckets), len(b.params))
                b.params.append(p)
                b.offsets.append(b.numel)
                b.numel += p.numel()
            self.buckets.append(b)
        self._next = 0
        self._hooks = []
        if self.active:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self.reset()

    def reset(self):
        """Arm for the next backward."""
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
        self._next = 0
        self._tl = None
        if self.timing:  # t0: the step's start (every time below is after it)
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record()
            self._tl = {"t0": t0, "ready": [], "done": [], "end": None}

    def _flat(self, b, like):
        if b.flat is None:
            b.flat = torch.empty(b.numel, dtype=torch.float32, device=like.device)
        return b.flat

    def _on_grad(self, p):
        bi, k = self.where[p]
        b = self.buckets[bi]
        flat = self._flat(b, p)
        off = b.offsets[k]
        torch.mul(p.grad.reshape(-1), 1.0 / self.world, out=flat[off: off + p.numel()])
        b.pending -= 1
        self._launch_ready()

    def _launch_ready(self):
        while self._next < len(self.buckets) and self.buckets[self._next].pending == 0:
            b = self.buckets[self._next]
            if self.captured:
                # (the replay launches this bucket's all-reduce: launch_captured)
                self._events.append(self._next)
                self._next += 1
                continue
            tl = self._tl
            if tl is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                tl["ready"].append(ev)
            b.work = dist.all_reduce(b.flat, group=self.group, async_op=True)
            if tl is not None:
                # a side stream that waits on this collective alone: its event
                # marks the all-reduce's completion, not the compute stream's
                side = self._side_stream(b.flat.device)
                with torch.cuda.stream(side):
                    b.work.wait()
                    ev = torch.cuda.Event(enable_timing=True)
                    ev.record(side)
                tl["done"].append(ev)
            self._next += 1

    def _side_stream(self, device):
        st = getattr(self, "_side", None)
        if st is None:
            st = self._side = torch.cuda.Stream(device=device)
        return st

    def begin_capture(self):
        """Arm the capture form for the backward about to be captured."""
        if self._flat_missing():
            raise RuntimeError("reducer: the buckets must exist before a capture (run an eager "
                               "step first)")
        self.reset()
        self.captured = True
        self._events = []

    def end_capture(self):
        """The buckets completed in the capture just finished, in order."""
        events, self._events, self.captured = self._events, None, False
        if len(events) != len(self.buckets):
            raise RuntimeError(f"reducer: {len(events)} of {len(self.buckets)} buckets became "
                               "ready in the capture")
        return events

    def _flat_missing(self):
        return any(b.flat is None for b in self.buckets)

    def launch_captured(self, events):
        """At a replay, after the captured backward was launched (on the
        current stream): every bucket's all-reduce, in order, on the side
        stream after it."""
        side = self._side_stream(self.buckets[0].flat.device)
        side.wait_stream(torch.cuda.current_stream(side.device))
        with torch.cuda.stream(side):
            for bi in events:
                b = self.buckets[bi]
                b.work = dist.all_reduce(b.flat, group=self.group, async_op=True)

    def wait_captured(self):
        """The current stream waits for every bucket's all-reduce."""
        for b in self.buckets:
            b.work.wait()
            b.work = None

    def finish(self):
        """Wait for every bucket and expose the averaged gradients as .grad.
        In the capture form: no wait (the replay launches the collectives,
        launch_captured); the gradients become views of the buckets."""
        if not self.active:
            return
        if self.captured:
            for b in self.buckets:
                if b.pending:
                    for p, off in zip(b.params, b.offsets):
                        if p.grad is None:
                            b.flat[off: off + p.numel()].zero_()
                    b.pending = 0
            self._launch_ready()
            for b in self.buckets:
                for p, off in zip(b.params, b.offsets):
                    p.grad = b.flat[off: off + p.numel()].view_as(p)
            return
        if self._tl is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._tl["end"] = ev
        for b in self.buckets:
            if b.pending:
                # a parameter got no gradient this step: contribute zeros (all ranks
                # take the same branch because the graph is the same on every rank)
                flat = self._flat(b, b.params[0])
                for p, off in zip(b.params, b.offsets):
                    if p.grad is None:
                        flat[off: off + p.numel()].zero_()
                b.pending = 0
        self._launch_ready()
        for b in self.buckets:
            b.work.wait()
            for p, off in zip(b.params, b.offsets):
                p.grad = b.flat[off: off + p.numel()].view_as(p)
        self.last_timeline = self._tl
        self.reset()

    def timeline(self):
        """Per-bucket ready / done times (ms, relative to the end of backward;
        negative = before it) of the last timed step, the all-reduce time left
        exposed after backward (``exposed_ms`` = last completion - end of
        backward, >= 0) and the collectives' busy time (each bucket from
        max(its ready time, the previous completion) to its completion).
        Synchronises; None if no step was timed."""
        tl = getattr(self, "last_timeline", None)
        if not tl or tl["end"] is None or not tl["done"]:
            return None
        torch.cuda.synchronize()
        t0 = tl["t0"]
        end = t0.elapsed_time(tl["end"])
        ready = [t0.elapsed_time(e) - end for e in tl["ready"]]
        done = [t0.elapsed_time(e) - end for e in tl["done"]]
        busy, prev = 0.0, float("-inf")
        for r, d in zip(ready, done):
            busy += max(0.0, d - max(r, prev))
            prev = d
        exposed = max(0.0, done[-1])
        return {"buckets": len(done),
                "bucket_mb": [round(b.numel * 4 / 2 ** 20, 2) for b in self.buckets],
                "ready_ms_vs_backward_end": [round(v, 3) for v in ready],
                "done_ms_vs_backward_end": [round(v, 3) for v in done],
                "step_start_to_backward_end_ms": round(end, 3),
                "exposed_ms": round(exposed, 3), "busy_ms": round(busy, 3),
                "hidden_frac": round(1.0 - exposed / busy, 4) if busy > 0 else None}

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
