#!/usr/bin/env python
"""Runs tests/rccl_worker.py (two Trainer.steps with and without the RCCL
reducer, which must give bit-identical parameters) once per environment
setting, one child process after another, and prints the max parameter
difference of each: which kernel-selection switch the equality depends on."""
import os
import socket
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARMS = [("default", {}), ("conv_stream=0", {"D2MI_CONV_STREAM": "0"}),
        ("conv_stream_nt=0", {"D2MI_CONV_STREAM_NT": "0"}),
        ("rpn_merge=0", {"D2MI_RPN_MERGE": "0"}), ("roi_bwd_rec=0", {"D2MI_ROI_BWD_REC": "0"}),
        ("roi_heavy=0", {"D2MI_ROI_HEAVY": "0"}), ("nms_scan=0", {"D2MI_NMS_SCAN": "0"}),
        ("rpn_compact=0", {"D2MI_RPN_COMPACT": "0"}), ("default again", {})]
if len(sys.argv) > 1:  # a subset by name
    ARMS = [a for a in ARMS if a[0] in sys.argv[1:]]



def port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


for name, extra in ARMS:
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port()), RANK="0",
                   WORLD_SIZE="1", LOCAL_RANK="0", OMP_NUM_THREADS="4", **extra)
        p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_worker.py"), d],
                           env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=300)
        if p.returncode != 0:
            print(f"{name}: worker exit {p.returncode}\n{p.stdout[-2000:]}", flush=True)
            sys.exit(1)
        r = torch.load(os.path.join(d, "rccl.pt"), weights_only=True)
        diff = (r["rccl"] - r["plain"]).abs()
        nz = int((diff > 0).sum())
        print(f"{name}: max |rccl - plain| = {diff.max().item():.3g} over {nz} params; losses equal "
              f"{r['rccl_losses'] == r['plain_losses']}", flush=True)
