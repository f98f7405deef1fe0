#!/usr/bin/env python
"""Instruction-fetch cost of one-shot straight-line code (tools/icache_probe.hip).

Builds the probe library (hipcc, gfx950) next to this script on first use,
then for straight-line bodies of 256 / 1,024 / 4,096 unrolled FMA pairs (and
the same work as a rolled loop) prints the kernel's own wall time, cold (after
a kernel that streams 1 GiB) and warm (launched again at once), with the code
size of each kernel from the code object.

    python tools/icache_probe.py
"""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "icache_probe.hip")
LIB = os.path.join(HERE, "libicache_probe.so")


def build():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared",
                               "-fPIC", SRC, "-o", LIB])
    return ctypes.CDLL(LIB)


def main():
    lib = build()
    if not torch.cuda.is_available():
        print("built", LIB)
        return
    dev = torch.device("cuda:0")
    out = torch.zeros(1 << 16, device=dev)
    t = torch.zeros(2, dtype=torch.int64, device=dev)
    big = torch.ones(1 << 28, device=dev)  # 1 GiB
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    vp = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731

    def run(launch):
        res = {}
        for mode in ("cold", "warm"):
            vals = []
            for _ in range(5):
                if mode == "cold":
                    lib.probe_stream(vp(big), vp(out), ctypes.c_size_t(big.numel()), st)
                else:
                    launch()
                launch()
                torch.cuda.synchronize()
                a, b = t.tolist()
                vals.append((b - a) / 100.0)
            vals.sort()
            res[mode] = vals[len(vals) // 2]
        return res

    for which, n in enumerate((256, 1024, 4096)):
        r = run(lambda: lib.probe_straight(which, vp(out), vp(t), st))
        ro = run(lambda: lib.probe_rolled(n, vp(out), vp(t), st))
        print(f"{n:5d} FMA pairs: straight-line (~{n * 16 / 1024:.0f} KB of code) cold {r['cold']:7.2f} us"
              f" warm {r['warm']:7.2f} us | rolled loop cold {ro['cold']:7.2f} us warm {ro['warm']:7.2f} us",
              flush=True)


if __name__ == "__main__":
    sys.exit(main())
