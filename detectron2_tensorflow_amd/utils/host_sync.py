"""The hot path's few host synchronisations, timed.

Every place where the host must read a device value before it can size the
next launches (the mask branch's foreground count, a SOLOv2 image's live
cells) goes through ``read_ints``: it returns the values and adds the time
the host spent blocked on the device to ``blocked_s``.  tools/host_time.py
subtracts that from the step's host time to report the host's own enqueue
work (Python + launches), which is what bounds a launch-bound step.
"""
import time

import torch

blocked_s = 0.0


def read_ints(t):
    """int values of a small device tensor (one synchronising copy)."""
    global blocked_s
    t0 = time.perf_counter()
    if t.is_cuda:
        torch.cuda.current_stream(t.device).synchronize()
    t1 = time.perf_counter()
    blocked_s += t1 - t0
    return [int(v) for v in t.reshape(-1).cpu().tolist()]


def arm_pinned(host):
    """Mark a pinned int64 host buffer unwritten (-1) before the work that
    writes it is queued (read_pinned spins on it)."""
    host.fill_(-1)


def read_pinned(host, spin_s=0.005):
    """int values of a pinned host tensor that the work queued on the current
    stream writes (a captured graph's last copy), armed by arm_pinned: the
    host spins on the buffer itself for up to ``spin_s`` (a blocking stream
    wait wakes the host tens of microseconds after the copy lands), then
    waits on the stream (timed either way; the wait also surfaces a device
    error the spin cannot see)."""
    global blocked_s
    t0 = time.perf_counter()
    view = host.numpy()
    while view[0] < 0 and time.perf_counter() - t0 < spin_s:
        pass
    if view[0] < 0:
        torch.cuda.current_stream().synchronize()
    blocked_s += time.perf_counter() - t0
    return [int(v) for v in view.tolist()]


class PendingRead:
    """A device-to-host read started early: the values are copied into pinned
    host memory behind the work already queued, an event marks them ready,
    and the host keeps enqueueing until it actually needs them."""

    def __init__(self, t):
        self.host = torch.empty(t.numel(), dtype=t.dtype, pin_memory=True)
        self.host.copy_(t.reshape(-1), non_blocking=True)
        self.event = torch.cuda.Event()
        self.event.record(torch.cuda.current_stream(t.device))


def start_read(t):
    """Begin reading a small device tensor without blocking (finish_read)."""
    if not t.is_cuda:
        return [int(v) for v in t.reshape(-1).tolist()]
    return PendingRead(t)


def finish_read(p):
    """int values of a start_read, blocking (and timed) only if not yet there."""
    global blocked_s
    if not isinstance(p, PendingRead):
        return p
    t0 = time.perf_counter()
    p.event.synchronize()
    blocked_s += time.perf_counter() - t0
    return [int(v) for v in p.host.tolist()]


def reset():
    global blocked_s
    blocked_s = 0.0
