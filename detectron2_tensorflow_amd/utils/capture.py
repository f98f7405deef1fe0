"""Host tables for launches captured into a hipGraph (engine/graphed.py).

Some launches read a small per-call table from device memory (the fused
Momentum-SGD's tensor table, the batched FrozenBN fold's entries).  Eagerly
they are uploaded through a ring of pinned buffers, synchronised by events:
inside a capture that is not allowed (no event query, no pinned-buffer
reuse), and one device buffer per call site would be shared by every graph.
While a capture is in progress ``table`` hands out a FRESH slice of the
capture's table arena for the launch to read and queues the host bytes;
``flush`` fills the queued slices once the capture has ended (ordinary
synchronous copies) and hands the arena to the graph's owner to keep alive --
the table is constant across replays, since a graph's tensors never move.

Why an arena reserved BEFORE the capture (r5; the cause of the r4 replay
faults).  A table is written once, by the host, after the capture; nothing
inside the graph writes it.  Memory the caching allocator hands out DURING a
capture comes from the graph's private pool, and that pool reuses blocks in
stream order: a block freed earlier in the same capture (a temporary of an
earlier captured kernel), or freed by an earlier capture that shares the pool
(graph A's temporaries, reused by a B[R] graph), is handed out again.  Stream
order protects values that captured kernels produce, not bytes the host
wrote outside the graph: at replay the earlier kernel writes its temporary
over the table, and the launch that reads the table next takes garbage
pointers -- the illegal-address faults of r4 (graph A's fold table, a B[R]
graph's fold-backward / optimizer tables).  The arena is allocated outside
any capture, from the ordinary pool, and no captured temporary can land in
it.  ``tools/graph_audit.py`` proves both halves on the GPU without replaying
(allocator trace: every table slice against every earlier allocation).
"""
import numpy as np
import torch

_pending = []
_arena = None        # [device tensor, next free offset] while a capture may issue tables
ARENA_BYTES = 1 << 20
ALIGN = 256
# (tools/graph_audit.py) every table handed out: (address, nbytes, label); and a switch
# that restores the r4 behaviour (tables from the capture pool) for the audit's
# "before" half -- never for a replay
issued = []
ARENA = True


def capturing():
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def begin(device, nbytes=None):
    """Reserve the device memory the next capture's tables will live in.
    Must run OUTSIDE the capture (it allocates from the ordinary pool)."""
    global _arena
    if capturing():
        raise RuntimeError("capture.begin inside a capture: the table arena must be reserved "
                           "before the capture starts")
    n = int(nbytes or ARENA_BYTES)
    _arena = [torch.empty(n, dtype=torch.uint8, device=device), 0]


def table(arr, device, what="table"):
    """Device buffer for the host table ``arr`` (any numpy array) read by a
    launch being captured; filled by ``flush`` after the capture.  ``what``
    labels it for tools/graph_audit.py."""
    host = np.ascontiguousarray(arr).view(np.uint8).reshape(-1).copy()
    n = max(host.size, 1)
    if not ARENA:
        dev = torch.empty(n, dtype=torch.uint8, device=device)
    else:
        if _arena is None:
            raise RuntimeError("capture.table without capture.begin(): a table allocated from "
                               "the capture's own pool can be overwritten by a captured "
                               "temporary at replay")
        buf, off = _arena
        if buf.device != torch.device(device):
            raise RuntimeError(f"capture.table: arena on {buf.device}, table for {device}")
        if off + n > buf.numel():
            raise RuntimeError(f"capture table arena exhausted ({buf.numel()} bytes): pass a "
                               "larger size to capture.begin")
        dev = buf[off:off + n]
        _arena[1] = off + -(-n // ALIGN) * ALIGN
    issued.append((dev.data_ptr(), n, what))
    _pending.append((dev, host))
    return dev


def flush(keep):
    """Fill every table queued since the last flush (outside any capture) and
    append the device buffers (and the arena) to ``keep``."""
    global _arena
    if capturing():
        raise RuntimeError("capture.flush inside a capture")
    for dev, host in _pending:
        dev[:host.size].copy_(torch.from_numpy(host))
        keep.append(dev)
    _pending.clear()
    if _arena is not None:
        keep.append(_arena[0])
        _arena = None


def discard():
    """Drop the tables of an abandoned capture."""
    global _arena
    _pending.clear()
    _arena = None
