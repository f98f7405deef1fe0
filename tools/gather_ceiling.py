"""ROIAlign forward against the gather ceiling of its own access pattern (run
on the GPU box; verdict r3 item 4).

Runs the bench workload (Mask R-CNN R50-FPN training, 2 x 1333x800) for a few
steps, captures the LAST step's box-pooler inputs (p2..p5, the 1,024 sampled
ROIs), then times on them, interleaved, median of rounds:
  roi_align   the d2mi ROIAlign forward (what the step runs);
  gather4     tools/gather_ceiling.hip: the SAME 4 corner rows per bin (1 KiB
              each, the kernel's clamped taps, ROI-major bin order) read and
              summed into one output row -- the access pattern with the
              arithmetic removed: the ceiling for this launch's memory traffic;
  gather1_u   each distinct row read once (sorted), one 1 KiB row per output;
  copy        a streaming copy of the unique bytes (the HBM reference).
GB/s on the unique-bytes model (distinct rows + the output), as bench.py.

    python tools/gather_ceiling.py [--steps 4] [--iters 50] [--rounds 5]
"""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.path.join(ROOT, "tools", "libgather_ceiling.so")


def load_lib():
    src = os.path.join(ROOT, "tools", "gather_ceiling.hip")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["hipcc", "-O3", "-std=c++17", "-fPIC", "-shared",
                               "--offload-arch=gfx950", os.path.join(ROOT, "tools", "gather_ceiling.hip"),
                               "-o", LIB])
    lib = ctypes.CDLL(LIB)
    P, I = ctypes.c_void_p, ctypes.c_int
    lib.gc_gather4.argtypes = [P, P, I, P, I, P]
    lib.gc_gather1.argtypes = [P, P, I, P, P]
    lib.gc_copy.argtypes = [P, ctypes.c_longlong, P, P]
    lib.gc_copy_u.argtypes = [P, ctypes.c_longlong, P, I, I, P]
    lib.gc_gather1_u.argtypes = [P, P, I, P, I, I, P]
    lib.gc_gather_s.argtypes = [P, P, I, I, P, I, I, P]
    lib.gc_gather4_s.argtypes = [P, P, I, P, I, I, I, P]
    return lib


def corner_rows(boxes, box_ind, params, shapes):
    """[R * bins, 4] global row ids (levels concatenated) of the 4 corner rows
    the kernel loads per bin (S = 1; clamped taps, invalid samples included:
    the kernel's loads are unconditional), ROI-major then bin order."""
    import math
    (oh, ow, scales, sr, mode, pad, assign, min_l, max_l, canon_s, canon_l, _) = params
    dev = boxes.device
    b = boxes.detach().float().reshape(-1, 4)
    if assign and len(shapes) > 1:
        area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
        v = canon_l + torch.log(torch.sqrt(area) / canon_s + 2.220446049250313e-16) / math.log(2)
        lv = torch.nan_to_num(torch.floor(v), nan=min_l).clamp(min_l, max_l).long() - min_l
    else:
        lv = torch.zeros(b.shape[0], dtype=torch.long, device=dev)
    Hs = torch.tensor([s[1] for s in shapes], device=dev)[lv]
    Ws = torch.tensor([s[2] for s in shapes], device=dev)[lv]
    sc = torch.tensor(list(scales), dtype=torch.float32, device=dev)[lv]
    y1, x1, y2, x2 = (b * sc[:, None]).unbind(1)
    Hp, Wp = Hs + 2, Ws + 2
    y1, x1, y2, x2 = y1 + 1, x1 + 1, y2 + 1, x2 + 1
    i0, i1 = (Hp - 1).float(), (Wp - 1).float()
    sh, sw = (y2 - y1) / oh, (x2 - x1) / ow
    ny, nx = (y1 + sh / 2 - 0.5) / i0, (x1 + sw / 2 - 0.5) / i1
    y1, x1, y2, x2 = ny, nx, ny + sh * (oh - 1) / i0, nx + sw * (ow - 1) / i1

    def taps(c1, c2, img_p, img, crop):
        i = torch.arange(crop, device=dev, dtype=torch.float32)
        pos = c1[:, None] * (img_p - 1).float()[:, None] + i * ((c2 - c1) * (img_p - 1).float() / (crop - 1))[:, None]
        lo, hi = torch.floor(pos).long(), torch.ceil(pos).long()
        top = img[:, None] - 1
        return (lo - 1).clamp(min=0).minimum(top), (hi - 1).clamp(min=0).minimum(top)

    ylo, yhi = taps(y1, y2, Hp, Hs, oh)
    xlo, xhi = taps(x1, x2, Wp, Ws, ow)
    n = box_ind.detach().long().reshape(-1)
    base = torch.tensor([0] + [s[0] * s[1] * s[2] for s in shapes], device=dev).cumsum(0)
    img0 = (base[lv] + n * Hs * Ws)[:, None, None]
    rows = [img0 + yy[:, :, None] * Ws[:, None, None] + xx[:, None, :]
            for yy in (ylo, yhi) for xx in (xlo, xhi)]  # corner order 00, 01, 10, 11
    return torch.stack([r.reshape(-1) for r in rows], 1).to(torch.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    from detectron2_tensorflow_amd import _C
    from detectron2_tensorflow_amd.layers import ops
    import bench
    _C.load()
    dev = torch.device("cuda:0")
    args = argparse.Namespace(model="mask_rcnn_R_50_FPN", mode="train", batch=2, height=800,
                              width=1333, gpus=1, mask_format="raw")
    cfg, model = bench.build(args, dev)
    batch = bench.synthetic_batch(args, dev, 0)
    bench.calibrate_scores(model, batch)
    from detectron2_tensorflow_amd.engine import Trainer
    trainer = Trainer(cfg, model)
    cap = {}
    real = ops.roi_align

    def spy(features, boxes, box_ind, output_size, scales, *rest, **kw):
        if output_size in (7, (7, 7)):
            cap["in"] = ([f.detach() for f in features], boxes.detach().clone(),
                         box_ind.detach().clone(), output_size, scales, rest, dict(kw))
        return real(features, boxes, box_ind, output_size, scales, *rest, **kw)

    ops.roi_align = spy
    for _ in range(a.steps):
        trainer.step(batch)
    ops.roi_align = real
    torch.cuda.synchronize()
    feats, boxes, box_ind, osz, scales, rest, kw = cap["in"]
    kw.pop("grad_share", None)
    run_roi = lambda: ops.roi_align(feats, boxes, box_ind, osz, scales, *rest, **kw)  # noqa: E731
    y = run_roi()
    L = len(feats)
    params = (7, 7, tuple(float(s) for s in scales), 0, ops.BOX_MODE_ALIGNED, 1, int(L > 1),
              2, 5, 224, 4, False)
    shapes = [tuple(f.shape) for f in feats]
    idx = corner_rows(boxes, box_ind, params, shapes).contiguous()
    nb = idx.shape[0]
    C = feats[0].shape[-1]
    assert C == 256 and nb == y.shape[0] * 49
    src = torch.cat([f.reshape(-1, C) for f in feats]).contiguous()
    uniq = torch.unique(idx.long()).to(torch.int32)
    out4 = torch.empty(nb, C, device=dev)
    out1 = torch.empty(uniq.numel(), C, device=dev)
    lib = load_lib()
    st = _C.stream_of(dev)
    ub = (uniq.numel() + nb) * C * 4  # unique-bytes model (rows read + output written)
    cb = uniq.numel() * C * 4
    cp_src = src[:uniq.numel()].contiguous()
    cp_out = torch.empty_like(cp_src)
    def roi_tv(v):
        def fn():
            old = ops.get_tuning("roi_fwd")
            ops.set_tuning("roi_fwd", v)
            try:
                run_roi()
            finally:
                ops.set_tuning("roi_fwd", old)
        return fn

    arms = {
        "roi_align": run_roi,
        # r6: one wave iteration per wave (bit 16), U = 4 / 2 / 8 bins in flight
        "roi_align_1it_u4": roi_tv(2 | 4 | 8 | 16),
        "roi_align_1it_u2": roi_tv(1 | 2 | 4 | 8 | 16),
        "roi_align_1it_u8": roi_tv(2 | 4 | 8 | 16 | 32),
        # r6: corner rows loaded non-temporally (bit 64)
        "roi_align_ntl_u2": roi_tv(1 | 2 | 4 | 8 | 64),
        "roi_align_ntl_u4": roi_tv(2 | 4 | 8 | 64),
        "roi_align_ntl_1it_u4": roi_tv(2 | 4 | 8 | 16 | 64),
        # r6: the forward's 4-corner pattern in the guide's shape (scalar
        # corner indices, persistent 16 waves per CU), default / nt loads
        "gather4_s_u2": lambda: lib.gc_gather4_s(src.data_ptr(), idx.data_ptr(), nb, out4.data_ptr(),
                                                 2, 0, 1024, st),
        "gather4_s_u4": lambda: lib.gc_gather4_s(src.data_ptr(), idx.data_ptr(), nb, out4.data_ptr(),
                                                 4, 0, 1024, st),
        "gather4_s_u2_nt": lambda: lib.gc_gather4_s(src.data_ptr(), idx.data_ptr(), nb,
                                                    out4.data_ptr(), 2, 1, 1024, st),
        "gather4_u4": lambda: lib.gc_gather4(src.data_ptr(), idx.data_ptr(), nb, out4.data_ptr(), 4, st),
        "gather4_u2": lambda: lib.gc_gather4(src.data_ptr(), idx.data_ptr(), nb, out4.data_ptr(), 2, st),
        "gather1_unique": lambda: lib.gc_gather1(src.data_ptr(), uniq.data_ptr(), uniq.numel(),
                                                 out1.data_ptr(), st),
        "copy_unique_bytes": lambda: lib.gc_copy(cp_src.data_ptr(), cb // 16, cp_out.data_ptr(), st),
        # r5: unrolled forms (U loads in flight per lane, persistent grid)
        "gather1_unique_u8": lambda: lib.gc_gather1_u(src.data_ptr(), uniq.data_ptr(), uniq.numel(),
                                                      out1.data_ptr(), 8, 2048, st),
        "copy_unique_u8": lambda: lib.gc_copy_u(cp_src.data_ptr(), cb // 16, cp_out.data_ptr(), 8,
                                                2048, st),
    }
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)  # > the 256 MiB MALL

    def timeit(fn, cold=True):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        tot = 0.0
        for _ in range(a.iters):
            if cold:
                flush.zero_()  # cold caches
            else:
                # warm: the maps rewritten just before, as the FPN writes them in
                # the step (they then sit in the MALL / L2 as far as they fit)
                for f in feats:
                    f.add_(0.0)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            tot += e0.elapsed_time(e1)
        return tot / a.iters * 1e3

    for v in (2 | 4 | 8 | 16, 1 | 2 | 4 | 8 | 16, 2 | 4 | 8 | 16 | 32, 1 | 2 | 4 | 8 | 64,
              2 | 4 | 8 | 64, 2 | 4 | 8 | 16 | 64):
        old = ops.get_tuning("roi_fwd")
        ops.set_tuning("roi_fwd", v)
        try:
            yv = run_roi()
        finally:
            ops.set_tuning("roi_fwd", old)
        print(f"roi_fwd variant {v}: output equal to the default's: {bool(torch.equal(yv, y))}",
              flush=True)
    copy_validation(lib, dev, st)
    guide_gather(lib, dev, st, uniq, src, C, flush, a.iters)
    t = {k: [] for k in arms}
    tw = {k: [] for k in arms}
    for _ in range(a.rounds):
        for k, fn in arms.items():
            t[k].append(timeit(fn))
            tw[k].append(timeit(fn, cold=False))
    med = {k: statistics.median(v) for k, v in t.items()}
    medw = {k: statistics.median(v) for k, v in tw.items()}
    print(f"box pooler of the step: {y.shape[0]} ROIs x 49 bins, {uniq.numel()} distinct rows "
          f"({cb / 1e6:.1f} MB), unique-bytes model {ub / 1e6:.1f} MB; cold caches per launch")
    for k, us in med.items():
        by = (cb * 2 if k.startswith("copy_unique") else
              cb + uniq.numel() * C * 4 if k.startswith("gather1_unique") else ub)
        uw = medw[k]
        print(f"{k:20s} cold {us:7.1f} us {by / us / 1e3:7.1f} GB/s ({by / us / 1e3 / 8000:.3f})"
              f"  roi/this {med['roi_align'] / us:.3f} | maps-rewritten {uw:7.1f} us "
              f"{by / uw / 1e3:7.1f} GB/s ({by / uw / 1e3 / 8000:.3f}) roi/this "
              f"{medw['roi_align'] / uw:.3f}", flush=True)


def guide_gather(lib, dev, st, uniq, src, C, flush, iters):
    """r6 (verdict r5 weak #3): the guide's register gather (MI355X_MICROARCH.md
    'Indexed rows', last paragraph: random whole 1,152-B rows of a buffer far
    larger than the Infinity Cache, each fetched once, one wave per
    destination, 4 rows in flight, 16 waves per CU: 5.5-5.6 TB/s) with
    wave-uniform scalar row indices (gather_s_kernel), then the same kernel on
    the box pooler's own distinct rows, cold and warm."""
    rows = 2 << 20  # 2 GiB of 1 KiB rows (8x the 256 MiB Infinity Cache)
    table = torch.empty(rows * C, device=dev)
    perm = torch.randperm(rows, device=dev).to(torch.int32)
    grid = 256 * 4  # 4 workgroups of 4 waves per CU: 16 waves per CU
    out_sum = torch.empty(rows // 4 + 1, C, device=dev)
    out_copy = torch.empty(rows, C, device=dev)

    def t_of(fn, cold, n_it):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        fn()
        for _ in range(n_it):
            if cold:
                flush.zero_()
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return statistics.median(ts)

    for u in (4, 8):
        for mode in (1, 0):
            out = out_sum if mode else out_copy
            us = t_of(lambda: lib.gc_gather_s(table.data_ptr(), perm.data_ptr(), rows, mode,
                                              out.data_ptr(), u, grid, st), False, 5)
            rd = rows * C * 4
            wr = (rows // u if mode else rows) * C * 4
            print(f"guide gather 2 GiB table, random rows once, U={u} "
                  f"{'sum (1 row written per U)' if mode else 'copy (every row written)'}: "
                  f"{us:9.1f} us  read {rd / us / 1e3:7.1f} GB/s  read+write "
                  f"{(rd + wr) / us / 1e3:7.1f} GB/s", flush=True)
    del table, out_copy
    # the pooler's distinct rows (their own addresses in the concatenated levels)
    n = uniq.numel()
    shuf = uniq[torch.randperm(n, device=dev)].contiguous()
    out1 = torch.empty(n, C, device=dev)
    for order, ids in (("sorted", uniq), ("shuffled", shuf)):
        for cold in (True, False):
            for mode in (1, 0):
                us = t_of(lambda: lib.gc_gather_s(src.data_ptr(), ids.data_ptr(), n, mode,
                                                  out1.data_ptr(), 4, grid, st), cold, iters)
                rd = n * C * 4
                wr = (n // 4 if mode else n) * C * 4
                print(f"pooler rows ({n}, {rd / 1e6:.1f} MB) {order:8s} {'cold' if cold else 'warm'} "
                      f"{'sum ' if mode else 'copy'} U=4: {us:8.1f} us  read {rd / us / 1e3:7.1f} GB/s"
                      f"  read+write {(rd + wr) / us / 1e3:7.1f} GB/s", flush=True)


def copy_validation(lib, dev, st, iters=20):
    """The unrolled copy on a 1 GiB buffer (the guide's streaming-copy
    measurement, MI355X_MICROARCH.md: 6.29 TB/s) and at the pooler's size:
    validates the ceiling kernel itself before it is used as one."""
    for mb in (1024, 134):
        n4 = (mb << 20) // 16
        a_ = torch.empty(n4 * 4, device=dev)
        b_ = torch.empty_like(a_)
        for name, fn in (("copy (r4, 1 float4 / iteration)", lambda: lib.gc_copy(a_.data_ptr(), n4, b_.data_ptr(), st)),
                         ("copy_u8 (r5)", lambda: lib.gc_copy_u(a_.data_ptr(), n4, b_.data_ptr(), 8, 2048, st)),
                         ("copy_u4 (r5)", lambda: lib.gc_copy_u(a_.data_ptr(), n4, b_.data_ptr(), 4, 4096, st))):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                fn()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) / iters * 1e3
            print(f"validation {mb:5d} MiB {name:34s} {us:9.1f} us  "
                  f"{2 * (mb << 20) / us / 1e3:7.1f} GB/s (read + write)", flush=True)
        del a_, b_


if __name__ == "__main__":
    main()
