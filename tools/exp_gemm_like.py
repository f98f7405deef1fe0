import sys, os, math, json, torch
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
for name, N, H, W, Cin, Cout, k in [("gemm-like 1x1 K=2304", 2, 200, 336, 2304, 256, 1),
                                    ("fpn p2 3x3", 2, 200, 336, 256, 256, 3),
                                    ("1x1 K=2304 N=512", 2, 200, 336, 2304, 512, 1),
                                    ("1x1 K=1024 M=4096^2", 1, 64, 256, 4096, 4096, 1)]:
    x = torch.randn(N, H, W, Cin, device=dev)
    w = torch.randn(k, k, Cin, Cout, device=dev) / math.sqrt(k*k*Cin)
    wp = ops.pack_conv_weights(w)
    p = (k-1)//2
    ms = timeit(lambda: ops.conv2d_nhwc(x, wp, None, 1, (p, p)))
    fl = 2.0*N*H*W*Cout*k*k*Cin
    mm = None
    if k == 1:
        a2 = x.reshape(-1, Cin); b2 = w.reshape(Cin, Cout)
        mm = timeit(lambda: torch.mm(a2, b2))
    print(json.dumps({"shape": name, "us": round(ms*1e3,1), "tflops": round(fl/ms/1e9,1),
                      "hipblaslt_tflops": round(fl/mm/1e9,1) if mm else None}))
