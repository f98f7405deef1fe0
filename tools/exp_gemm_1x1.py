"""Experiment: backbone 1x1 convs — MFMA conv kernel vs hipBLASLt addmm (+ residual / ReLU passes)."""
import sys, math, json, torch
sys.path.insert(0, "/root/repo")
from detectron2_tensorflow_amd import _C
from detectron2_tensorflow_amd.layers import ops
_C.load()
dev = torch.device("cuda:0")
def timeit(fn, iters=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters
shapes = [("res2 conv3+res", 2, 200, 336, 64, 256, True), ("res2 conv1", 2, 200, 336, 256, 64, False),
          ("res3 conv1", 2, 100, 168, 512, 128, False), ("res3 conv3+res", 2, 100, 168, 128, 512, True),
          ("res4 conv1", 2, 50, 84, 1024, 256, False), ("res4 conv3+res", 2, 50, 84, 256, 1024, True),
          ("res5 conv1", 2, 25, 42, 2048, 512, False), ("res5 conv3+res", 2, 25, 42, 512, 2048, True),
          ("dgrad res4 conv3", 2, 50, 84, 1024, 256, False), ("fpn lat p2", 2, 200, 336, 256, 256, False)]
for name, N, H, W, Cin, Cout, res in shapes:
    x = torch.randn(N, H, W, Cin, device=dev)
    w = torch.randn(1, 1, Cin, Cout, device=dev) / math.sqrt(Cin)
    b = torch.randn(Cout, device=dev)
    r = torch.randn(N, H, W, Cout, device=dev) if res else None
    wp = ops.pack_conv_weights(w)
    ms1 = timeit(lambda: ops.conv2d_nhwc(x, wp, b, 1, (0, 0), relu=True, residual=r, relu_after_add=res))
    x2, w2, r2 = x.reshape(-1, Cin), w.reshape(Cin, Cout), (r.reshape(-1, Cout) if res else None)
    def gemm():
        if res:
            y = torch.addmm(r2, x2, w2)
            return y.add_(b).relu_()
        return torch.addmm(b, x2, w2).relu_()
    ms2 = timeit(gemm)
    ms3 = timeit(lambda: torch.mm(x2, w2))
    fl = 2.0 * N * H * W * Cin * Cout
    print(json.dumps({"shape": name, "mfma_us": round(ms1 * 1e3, 1), "gemm_epi_us": round(ms2 * 1e3, 1),
                      "mm_only_us": round(ms3 * 1e3, 1), "mfma_tf": round(fl / ms1 / 1e9, 1),
                      "mm_tf": round(fl / ms3 / 1e9, 1)}))
