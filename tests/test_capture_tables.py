"""utils/capture.py host tables (CPU): the r5 fix of the hipGraph replay
faults puts every table a captured launch reads into an arena reserved
BEFORE the capture (tools/graph_audit.py proves the overlap it removes on the
GPU).  Here the arena's bookkeeping: tables are disjoint, aligned slices of
the arena, filled by flush with their host bytes, the arena is handed to the
graph's owner, exhaustion raises, and a table without begin() raises."""
import numpy as np
import pytest
import torch

from detectron2_tensorflow_amd.utils import capture


def test_tables_are_disjoint_aligned_slices_of_the_arena():
    capture.discard()
    capture.begin(torch.device("cpu"), nbytes=4096)
    arena = capture._arena[0]
    hosts = [np.arange(n, dtype=np.uint8) for n in (10, 300, 1, 256)]
    devs = [capture.table(h, torch.device("cpu"), what=f"t{i}") for i, h in enumerate(hosts)]
    base = arena.data_ptr()
    spans = []
    for d, h in zip(devs, hosts):
        off = d.data_ptr() - base
        assert off % capture.ALIGN == 0
        assert 0 <= off and off + h.size <= arena.numel()
        spans.append((off, off + max(h.size, 1)))
    spans.sort()
    for (a0, a1), (b0, _) in zip(spans, spans[1:]):
        assert a1 <= b0, "tables overlap"
    keep = []
    capture.flush(keep)
    for d, h in zip(devs, hosts):
        assert np.array_equal(d[:h.size].numpy(), h)
    assert any(k.data_ptr() == base for k in keep), "flush must hand the arena over"
    assert capture._arena is None and not capture._pending


def test_table_without_begin_or_past_the_arena_raises():
    capture.discard()
    with pytest.raises(RuntimeError, match="without capture.begin"):
        capture.table(np.zeros(4, np.uint8), torch.device("cpu"))
    capture.begin(torch.device("cpu"), nbytes=512)
    capture.table(np.zeros(300, np.uint8), torch.device("cpu"))
    with pytest.raises(RuntimeError, match="exhausted"):
        capture.table(np.zeros(300, np.uint8), torch.device("cpu"))
    capture.discard()
    assert capture._arena is None and not capture._pending
