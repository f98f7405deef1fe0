#!/bin/bash
# conv_epi A/B (register-stored split-K partials) on the GPU box
timeout -k 10 300 python -u tools/ws_ab.py --key conv_epi --arms 0,1 --set kxk,short_k --iters 20 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u tools/ab_inproc.py --switch conv_epi --blocks 6 --steps 10 2>&1 | grep -v amdgpu.ids | tail -2
