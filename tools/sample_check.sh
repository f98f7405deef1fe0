#!/bin/bash
# fused subsample on the GPU box: its test, the training / DP / model tests,
# the in-step A/B, the glue-site count.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "subsample or stem" 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_train.py tests/test_gpu_dp.py tests/test_gpu_model.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 10 300 python -u tools/ab_inproc.py --switch fused_sample --blocks 8 --steps 10 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
timeout -k 10 300 python -u tools/glue_sites.py --rows 40 > gpurun_out/glue_sites2.txt 2>&1 || exit 1
