#!/bin/bash
# round-3 A/Bs on the GPU box (in process): the WS conv kernel per shape and in
# the training step, the WS wgrad kernel per shape, the ROIAlign forward
# variants on the step's own ROIs, then the C5 tests
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ws_ab.py --arms 0,1,2 --set kxk,short_k --iters 20 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u tools/ws_ab.py --key wgrad_ws --arms 0,1,2 --set wgrad --iters 10 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u tools/ab_inproc.py --switch conv_ws --blocks 6 --steps 10 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 10 200 python -u tools/roi_ab.py --arms 0,1,2,4,8,3,9,15 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u -m pytest tests/test_solo.py -k c5 -q --timeout 200 --timeout-method thread 2>&1 | tail -3
