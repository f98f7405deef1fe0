#!/bin/bash
# MFMA stem conv on the GPU box: its tests, an isolated timing against the
# MIOpen conv, the in-step A/B, then the glue-site count.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "stem" 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 10 120 python -u - <<'PY' 2>&1 | grep -v amdgpu.ids || exit 1
import torch, torch.nn.functional as F
from detectron2_tensorflow_amd.layers import ops
dev = torch.device("cuda", 0)
x = torch.randn(2, 800, 1344, 3, device=dev) * 50
w = torch.randn(7, 7, 3, 64, device=dev) / 12
w3 = ops.stem_conv_weights(w)
wc = w.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last)
def t(fn, n=50):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3
a = t(lambda: ops.stem_conv(x, w3))
b = t(lambda: F.conv2d(x.permute(0, 3, 1, 2), wc, None, stride=2, padding=3))
print(f"stem conv 2x800x1344x3->64: MFMA {a:.1f} us, MIOpen {b:.1f} us")
PY
timeout -k 10 300 python -u tools/ab_inproc.py --switch stem_mfma --blocks 8 --steps 10 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
timeout -k 10 300 python -u tools/glue_sites.py --rows 70 > gpurun_out/glue_sites.txt 2>&1 || exit 1
