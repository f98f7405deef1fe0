"""Which torch (non-library) kernels an eager training step launches, and
from where: one eager Trainer step of the bench's model under torch.profiler,
the aten ops that launch device work grouped by Python stack, sorted by device
time.  Usage (GPU box): python tools/torch_op_census.py [bench.py flags]."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    args = bench.parse()
    device = torch.device("cuda", 0)
    from detectron2_tensorflow_amd import _C
    _C.load()
    cfg, model = bench.build(args, device)
    batch = bench.synthetic_batch(args, device, 0)
    bench.calibrate_scores(model, batch)
    from detectron2_tensorflow_amd.engine import Trainer
    trainer = Trainer(cfg, model)
    for _ in range(3):
        trainer.step(batch)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=True) as prof:
        trainer.step(batch)
        torch.cuda.synchronize()
    keep = ("aten::copy_", "aten::add", "aten::add_", "aten::fill_", "aten::zero_",
            "aten::threshold_backward", "aten::cat", "aten::div", "aten::sub", "aten::mul",
            "aten::where", "aten::clamp", "aten::scatter", "aten::gather", "aten::index",
            "aten::flip", "aten::sum", "aten::eq", "aten::sort", "aten::random_",
            "aten::constant_pad_nd", "aten::masked_fill_", "aten::index_put_")
    ev = [e for e in prof.key_averages(group_by_input_shape=True, group_by_stack_n=6)
          if e.key in keep and e.device_time_total > 0]
    ev.sort(key=lambda e: -e.device_time_total)
    total = sum(e.device_time_total for e in ev)
    print(f"torch ops with device time in one eager step: {total / 1e3:.1f} ms")
    for e in ev[:40]:
        t = e.device_time_total
        print(f"\n{t:8.1f} us  x{e.count:3d}  {e.key}  {e.input_shapes}")
        for fr in (e.stack or [])[:6]:
            print("      ", fr)


if __name__ == "__main__":
    main()
