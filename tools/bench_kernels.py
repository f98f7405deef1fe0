"""Per-kernel micro-benchmarks of the hot path on the MI355X (HIP-event timing).

    python tools/bench_kernels.py [--only conv,roi,nms,topk] [--iters 20]

conv: the MFMA implicit-GEMM kernel vs torch/MIOpen conv2d (channels_last) on
the FPN / RPN / mask-head / backbone shapes of Mask R-CNN R50-FPN at 1333x800
(batch 2), in TFLOP/s of algorithmic flops.  roi: multi-level ROIAlign in
algorithmic GB/s.  nms/topk: microseconds per call.
"""
import argparse
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from detectron2_tensorflow_amd import _C  # noqa: E402
from detectron2_tensorflow_amd.layers import ops  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters  # ms


CONV_SHAPES = [
    # name, N, H, W, Cin, Cout, k, stride
    ("fpn_out_p2 3x3", 2, 200, 336, 256, 256, 3, 1),
    ("fpn_lat_p2 1x1", 2, 200, 336, 256, 256, 1, 1),
    ("fpn_lat_p5 1x1", 2, 25, 42, 2048, 256, 1, 1),
    ("fpn_out_p5 3x3", 2, 25, 42, 256, 256, 3, 1),
    ("mask_fcn 3x3", 200, 14, 14, 256, 256, 3, 1),
    ("rpn_1x1 256->15", 2, 200, 336, 256, 15, 1, 1),
    ("res2_conv2 3x3", 2, 200, 336, 64, 64, 3, 1),
    ("res4_conv1 1x1", 2, 50, 84, 1024, 256, 1, 1),
    ("res3_conv2 3x3", 2, 100, 168, 128, 128, 3, 1),
    ("res2_conv3 1x1 +res", 2, 200, 336, 64, 256, 1, 1),
    ("res4_conv3 1x1 +res", 2, 50, 84, 256, 1024, 1, 1),
    ("fpn_lat_p2 1x1 +td", 2, 200, 336, 256, 256, 1, 1),
]


SHAPE_FILTER = None
NO_MIOPEN = False


def bench_conv(dev, iters):
    out = []
    for name, N, H, W, Cin, Cout, k, s in CONV_SHAPES:
        if SHAPE_FILTER and SHAPE_FILTER not in name:
            continue
        x = torch.randn(N, H, W, Cin, device=dev)
        w = torch.randn(k, k, Cin, Cout, device=dev) / math.sqrt(k * k * Cin)
        b = torch.randn(Cout, device=dev)
        wp = ops.pack_conv_weights(w)
        p = (k - 1) // 2
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        flops = 2.0 * N * OH * OW * Cout * k * k * Cin
        res = td = None
        if name.endswith("+res"):
            res = torch.randn(N, OH, OW, Cout, device=dev)
        if name.endswith("+td"):
            td = torch.randn(N, (OH + 1) // 2, (OW + 1) // 2, Cout, device=dev)
        run = lambda mm: ops.conv2d_nhwc(x, wp, b, s, (p, p), relu=res is not None,  # noqa: E731
                                         residual=res, topdown=td,
                                         relu_after_add=res is not None, math_mode=mm)
        ms = timeit(lambda: run("f32"), iters)
        ms_s = timeit(lambda: run("split"), iters)
        err = {}
        if N * H * W <= 140000:  # float64 reference on a slice of the batch
            n1 = 1 if N <= 2 else 8
            x64 = x[:n1].double().permute(0, 3, 1, 2)
            ref = F.conv2d(x64, w.double().permute(3, 2, 0, 1), b.double(), stride=s, padding=p)
            ref = ref.permute(0, 2, 3, 1)
            if td is not None:
                ref = ref + td[:n1].double().repeat_interleave(2, 1).repeat_interleave(2, 2)[:, :OH, :OW]
            if res is not None:
                ref = torch.relu(ref + res[:n1].double())
            sc = ref.abs().max().item()
            for mm in ("f32", "split"):
                err[mm] = float((run(mm)[:n1].double() - ref).abs().max() / sc)
        xc = x.permute(0, 3, 1, 2)
        wc = w.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last)
        ms_t = float("nan") if NO_MIOPEN else timeit(
            lambda: F.conv2d(xc, wc, b, stride=s, padding=p), iters)
        out.append({"kernel": "conv", "shape": name, "mfma_us": round(ms * 1e3, 1),
                    "mfma_tflops": round(flops / ms / 1e9, 1),
                    "split_us": round(ms_s * 1e3, 1), "split_tflops": round(flops / ms_s / 1e9, 1),
                    "max_rel_err_f32": err.get("f32"), "max_rel_err_split": err.get("split"),
                    "miopen_us": round(ms_t * 1e3, 1),
                    "miopen_tflops": round(flops / ms_t / 1e9, 1)})
    return out


def bench_wgrad(dev, iters):
    """Weight gradient: MFMA wgrad kernel vs torch.nn.grad.conv2d_weight (MIOpen)."""
    out = []
    for name, N, H, W, Cin, Cout, k, s in CONV_SHAPES:
        if Cout % 4 or "+" in name:
            continue
        x = torch.randn(N, H, W, Cin, device=dev)
        p = (k - 1) // 2
        OH, OW = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        dy = torch.randn(N, OH, OW, Cout, device=dev)
        flops = 2.0 * N * OH * OW * Cout * k * k * Cin
        ms = timeit(lambda: ops.conv2d_wgrad(x, dy, k, s, (p, p), math_mode="f32"), iters)
        ms_s = timeit(lambda: ops.conv2d_wgrad(x, dy, k, s, (p, p), math_mode="split"), iters)
        xc, dyc = x.permute(0, 3, 1, 2), dy.permute(0, 3, 1, 2)
        if k == 1:
            x2, dy2 = x.reshape(-1, Cin), dy.reshape(-1, Cout)
            ms_t = timeit(lambda: torch.mm(x2.t(), dy2), iters)
        else:
            ms_t = timeit(lambda: torch.nn.grad.conv2d_weight(xc, (Cout, Cin, k, k), dyc, s, p),
                          iters)
        ref = torch.nn.grad.conv2d_weight(xc, (Cout, Cin, k, k), dyc, s, p).permute(2, 3, 1, 0)
        err = float((ops.conv2d_wgrad(x, dy, k, s, (p, p), math_mode="f32") - ref).abs().max() /
                    ref.abs().max().clamp(min=1e-30))
        err_s = float((ops.conv2d_wgrad(x, dy, k, s, (p, p), math_mode="split") - ref).abs().max() /
                      ref.abs().max().clamp(min=1e-30))
        out.append({"kernel": "wgrad", "shape": name, "mfma_us": round(ms * 1e3, 1),
                    "mfma_tflops": round(flops / ms / 1e9, 1),
                    "miopen_us": round(ms_t * 1e3, 1),
                    "miopen_tflops": round(flops / ms_t / 1e9, 1), "max_rel_err": err,
                    "split_us": round(ms_s * 1e3, 1), "split_tflops": round(flops / ms_s / 1e9, 1),
                    "max_rel_err_split": err_s})
    return out


def bench_roi(dev, iters):
    """Forward and backward at the inference (2000 x 7x7, 200 x 14x14) and the
    training shapes (1024 sampled ROIs x 7x7, 64 foreground ROIs x 14x14).
    Algorithmic bytes per SURVEY 8d D4: fwd R*oh*ow*C*20, bwd R*oh*ow*C*36."""
    g = torch.Generator(device="cpu").manual_seed(0)
    feats = [torch.randn(2, 800 // s, 1344 // s, 256, generator=g).to(dev) for s in (4, 8, 16, 32)]
    out = []
    for R, o, bwd in ((2000, 7, False), (200, 14, False), (1024, 7, True), (64, 14, True)):
        c = torch.rand(R, 2, generator=g) * torch.tensor([800.0, 1333.0])
        sz = torch.exp(torch.rand(R, generator=g) * math.log(50) + math.log(16))
        boxes = torch.stack([c[:, 0] - sz / 2, c[:, 1] - sz / 2, c[:, 0] + sz / 2, c[:, 1] + sz / 2], 1).to(dev)
        bi = torch.randint(0, 2, (R,), generator=g, dtype=torch.int32).to(dev)
        ms = timeit(lambda: ops.roi_align(feats, boxes, bi, (o, o), [0.25, 0.125, 0.0625, 0.03125]), iters)
        byts = R * o * o * 256 * 20
        out.append({"kernel": "roi_align_fwd", "rois": R, "out": o, "us": round(ms * 1e3, 1),
                    "alg_GBps": round(byts / ms / 1e6, 1)})
        if bwd:
            fg = [f.clone().requires_grad_(True) for f in feats]
            y = ops.roi_align(fg, boxes, bi, (o, o), [0.25, 0.125, 0.0625, 0.03125])
            gy = torch.randn_like(y)
            ms = timeit(lambda: torch.autograd.grad(y, fg, gy, retain_graph=True), iters)
            byts = R * o * o * 256 * 36
            out.append({"kernel": "roi_align_bwd", "rois": R, "out": o, "us": round(ms * 1e3, 1),
                        "alg_GBps": round(byts / ms / 1e6, 1)})
    return out


def bench_paste(dev, iters):
    """Mask pasting at Mask R-CNN inference size: 2 images x 100 detections,
    28x28 masks onto the 800x1344 padded canvas ("conventional").  HBM-write
    bound: algorithmic bytes = the uint8 canvas + the f32 box masks read."""
    g = torch.Generator(device="cpu").manual_seed(3)
    D, H, W = 200, 800, 1344
    m = torch.rand(D, 28, 28, generator=g).to(dev)
    c = torch.rand(D, 2, generator=g) * torch.tensor([800.0, 1333.0])
    sz = torch.exp(torch.rand(D, 2, generator=g) * math.log(25) + math.log(16))
    boxes = torch.cat([c - sz / 2, c + sz / 2], 1)[:, [0, 1, 2, 3]].to(dev)
    ms = timeit(lambda: ops.paste_masks(m, boxes, (H, W)), iters)
    byts = D * H * W + m.numel() * 4
    return [{"kernel": "paste_masks", "detections": D, "canvas": [H, W], "us": round(ms * 1e3, 1),
             "alg_GBps": round(byts / ms / 1e6, 1)}]


def bench_nms(dev, iters):
    g = torch.Generator(device="cpu").manual_seed(1)
    out = []
    for S, n, mo in ((10, 1000, 1000), (10, 2000, 1000), (2, 5000, 100)):
        c = torch.rand(S * n, 2, generator=g) * 800
        sz = torch.rand(S * n, 2, generator=g) * 200 + 8
        b = torch.cat([c, c + sz], 1).to(dev)
        sc = torch.rand(S * n, generator=g).to(dev)
        off = torch.arange(0, (S + 1) * n, n, dtype=torch.int32, device=dev)
        ms = timeit(lambda: ops.nms_segments(b, sc, off, mo, 0.7, seg_capacity=n), iters)
        out.append({"kernel": "nms", "segments": S, "per_seg": n, "max_out": mo, "us": round(ms * 1e3, 1)})
    return out


def bench_topk(dev, iters):
    out = []
    for lens, k, sig in (([201600, 50400, 12600, 3150, 819] * 2, 1000, False),
                         ([12096000, 3024000, 756000, 189000, 47520] * 2, 1000, True)):
        x = torch.randn(sum(lens), device=dev)
        start = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)[:-1]), dtype=torch.int64, device=dev)
        ln = torch.tensor(lens, dtype=torch.int32, device=dev)
        ms = timeit(lambda: ops.topk_segments(x, start, ln, k, max(lens), sigmoid=sig), iters)
        out.append({"kernel": "topk", "total": sum(lens), "k": k, "sigmoid": sig, "us": round(ms * 1e3, 1),
                    "alg_GBps": round(4 * sum(lens) / ms / 1e6, 1)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="conv,wgrad,roi,paste,nms,topk")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shape", default=None, help="substring filter on conv shape names")
    ap.add_argument("--no-miopen", action="store_true")
    a = ap.parse_args()
    global SHAPE_FILTER, NO_MIOPEN
    SHAPE_FILTER = a.shape
    NO_MIOPEN = a.no_miopen
    _C.load()
    dev = torch.device("cuda:0")
    fns = {"conv": bench_conv, "wgrad": bench_wgrad, "roi": bench_roi, "paste": bench_paste,
           "nms": bench_nms,
           "topk": bench_topk}
    for name in a.only.split(","):
        for row in fns[name](dev, a.iters):
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
