"""Real-model data parallelism (lib/engine/model_deploy.py:203-205, :408-438):
two ranks of Mask R-CNN R50-FPN training on DIFFERENT batches through
engine/reducer.py's bucketed all-reduce hooks, which the training graph's
gradient hand-offs (RPN level accumulator, stage-output join, the merged
box / mask pooler backward) must all feed.  Each rank is a child process
(tests/dp_worker.py, started with subprocess: no exec of this process), both
on cuda:0 over gloo.

Asserts, after each of 2 steps: the replicas are bit-identical, and they
equal one process applying the averaged gradients of both batches
(the reference's mean of the per-clone losses) to the whole-step bar;
rank 1 (fewer GT boxes) ran its mask branch on a different row count.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_dp_two_ranks_real_model(dev, tmp_path):
    env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               OMP_NUM_THREADS="4")
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"),
                                       str(tmp_path)], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} exit {p.returncode}:\n{o[-4000:]}"
    load = lambda n: torch.load(os.path.join(tmp_path, n), weights_only=True)
    rows = []
    for s in range(2):
        r0, r1, one = load(f"rank0_step{s}.pt"), load(f"rank1_step{s}.pt"), load(f"single_step{s}.pt")
        assert torch.equal(r0["params"], r1["params"]), f"replicas diverged at step {s}"
        assert r0["losses"] != r1["losses"]  # the ranks trained on different batches
        rows.append((r0["mask_rows"], r1["mask_rows"]))
        d = (r0["params"] - one["params"]).abs()
        scale = one["params"].abs().max().item()
        print(f"step {s}: max |dp - single| = {d.max().item():.3g} (param scale {scale:.3g}); "
              f"mask rows {r0['mask_rows']} / {r1['mask_rows']}")
        assert d.max().item() <= 1e-5 * scale, d.max().item()
    # the mask branches ran on different (padded) foreground row counts
    assert any(a != b for a, b in rows), rows
