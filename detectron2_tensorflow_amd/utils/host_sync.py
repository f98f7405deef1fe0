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


def reset():
    global blocked_s
    blocked_s = 0.0
