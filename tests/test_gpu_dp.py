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


@pytest.mark.parametrize("arm", ["eager", "graphed"])
def test_dp_two_ranks_real_model(dev, tmp_path, arm):
    """arm "graphed" (r6): the ranks replay GraphedTrainer's graphs, the
    all-reduces launched between the backward graph and the update graph."""
    env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               OMP_NUM_THREADS="4")
    procs = []
    for r in range(2):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dp_worker.py"),
                                       str(tmp_path), arm], env=e, stdout=subprocess.PIPE,
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
    steps = {"eager": 2, "graphed": 3}[arm]
    for s in range(steps):
        r0, r1, one = load(f"rank0_step{s}.pt"), load(f"rank1_step{s}.pt"), load(f"single_step{s}.pt")
        assert torch.equal(r0["params"], r1["params"]), f"replicas diverged at step {s}"
        assert r0["losses"] != r1["losses"]  # the ranks trained on different batches
        rows.append((r0["mask_rows"], r1["mask_rows"]))
        d = (r0["params"] - one["params"]).abs()
        scale = one["params"].abs().max().item()
        print(f"step {s}: max |dp - single| = {d.max().item():.3g} (param scale {scale:.3g}); "
              f"mask rows {r0['mask_rows']} / {r1['mask_rows']}")
        if s < 2:
            # (a third step drifts further from the one-process sum order:
            # 4e-5 at step 2 on the eager replicas too, r6c)
            assert d.max().item() <= 1e-5 * scale, d.max().item()
        if arm == "graphed":
            # the graph-replayed replicas: bit-identical to the eager ones
            assert r0["replays"] == r1["replays"] == s, (s, r0["replays"], r1["replays"])
            for r in (r0, r1):
                assert torch.equal(r["graphed_params"], r["params"]), \
                    (s, float((r["graphed_params"] - r["params"]).abs().max()))
                assert r["graphed_losses"] == r["losses"], s
                assert r["graphed_rows"] == r["mask_rows"], s
    if arm == "graphed":
        census = load("rank0_step2.pt")["census"]
        print("rank 0 node census", census)
        assert "U" in census and all(c.get("memset", 0) == 0 for c in census.values())
    # the mask branches ran on different (padded) foreground row counts
    assert any(a != b for a, b in rows), rows


def test_rccl_backend_one_rank_runs_the_reducer(dev, tmp_path):
    """The "nccl" (RCCL) backend initialised in a fresh child process at
    world size 1 (tests/rccl_worker.py): three Trainer.steps of the real model
    with the bucketed all-reduce forced on give parameters bit-identical to
    the same steps without the reducer, and the timed step's per-bucket
    events form a consistent timeline (every bucket ready before it
    completes, the last completion no earlier than the end of backward
    minus nothing: exposed_ms >= 0).  r6: the same three steps through
    GraphedTrainer with the RCCL reducer (replayed graphs, the all-reduces
    launched between them) are bit-identical too."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0", OMP_NUM_THREADS="4")
    p = subprocess.Popen([sys.executable, os.path.join(HERE, "rccl_worker.py"), str(tmp_path)],
                         env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        out = p.communicate(timeout=240)[0]
    finally:
        if p.poll() is None:
            p.kill()
    assert p.returncode == 0, f"rccl worker exit {p.returncode}:\n{out[-4000:]}"
    res = torch.load(os.path.join(tmp_path, "rccl.pt"), weights_only=True)
    assert res["backend"] == "nccl"
    assert torch.equal(res["rccl"], res["plain"]), float((res["rccl"] - res["plain"]).abs().max())
    assert res["rccl_losses"] == res["plain_losses"]
    # r6: the graphed step over RCCL (2 replays after the eager warm-up)
    assert res["replays"] == 2 and "U" in res["census"], (res["replays"], res["census"])
    assert torch.equal(res["rccl_graphed"], res["plain"]), \
        float((res["rccl_graphed"] - res["plain"]).abs().max())
    assert res["rccl_graphed_losses"] == res["plain_losses"]
    tl = res["timeline"]
    print("rccl timeline:", tl)
    assert tl is not None and tl["buckets"] == res["buckets"] >= 5
    assert all(r <= d + 1e-3 for r, d in zip(tl["ready_ms_vs_backward_end"],
                                              tl["done_ms_vs_backward_end"]))
    assert tl["exposed_ms"] >= 0.0 and tl["busy_ms"] > 0.0
