#!/usr/bin/env python
"""Does a replayed hipGraph run independent branches concurrently?  Two spin
kernels (torch.cuda._sleep: one wave each) captured on two forked streams,
joined, replayed: ~T if the branches overlap, ~2T if the runtime serialises
them.  Also the same two spins captured on one stream (the serial
reference).  A diagnosis for a multi-stream capture of the training step
(weight gradients beside data gradients)."""
import sys

import torch


def main():
    cycles = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    dev = torch.device("cuda", 0)
    main_s = torch.cuda.Stream(device=dev)
    side = torch.cuda.Stream(device=dev)

    def body(fork):
        if fork:
            side.wait_stream(torch.cuda.current_stream())
            torch.cuda._sleep(cycles)
            with torch.cuda.stream(side):
                torch.cuda._sleep(cycles)
            torch.cuda.current_stream().wait_stream(side)
        else:
            torch.cuda._sleep(cycles)
            torch.cuda._sleep(cycles)

    res = {}
    for fork in (False, True):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(main_s):
            body(fork)  # warm
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=main_s):
                body(fork)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(5):
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        res["forked" if fork else "serial"] = sorted(ts)[2]
    # one spin alone, eager
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(cycles)
    e1.record()
    e1.synchronize()
    one = e0.elapsed_time(e1)
    print(f"one spin {one:.3f} ms; graph serial {res['serial']:.3f} ms; graph forked "
          f"{res['forked']:.3f} ms -> branches {'overlap' if res['forked'] < 1.5 * one else 'serialised'}",
          flush=True)


if __name__ == "__main__":
    main()
