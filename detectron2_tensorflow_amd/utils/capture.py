"""Host tables for launches captured into a hipGraph (engine/graphed.py).

Some launches read a small per-call table from device memory (the fused
Momentum-SGD's tensor table, the batched FrozenBN fold's entries).  Eagerly
they are uploaded through a ring of pinned buffers, synchronised by events:
inside a capture that is not allowed (no event query, no pinned-buffer
reuse), and one device buffer per call site would be shared by every graph.
While a capture is in progress ``table`` hands out a FRESH device buffer
(the capture's memory pool) for the launch to read and queues the host
bytes; ``flush`` fills the queued buffers once the capture has ended
(ordinary synchronous copies) and hands them to the graph's owner to keep
alive -- the table is constant across replays, since a graph's tensors never
move.
"""
import numpy as np
import torch

_pending = []


def capturing():
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def table(arr, device):
    """Device buffer for the host table ``arr`` (any numpy array) read by a
    launch being captured; filled by ``flush`` after the capture."""
    host = np.ascontiguousarray(arr).view(np.uint8).reshape(-1).copy()
    dev = torch.empty(max(host.size, 1), dtype=torch.uint8, device=device)
    _pending.append((dev, host))
    return dev


def flush(keep):
    """Fill every table queued since the last flush (outside any capture) and
    append the device buffers to ``keep``."""
    if capturing():
        raise RuntimeError("capture.flush inside a capture")
    for dev, host in _pending:
        dev[:host.size].copy_(torch.from_numpy(host))
        keep.append(dev)
    _pending.clear()


def discard():
    """Drop the tables of an abandoned capture."""
    _pending.clear()
