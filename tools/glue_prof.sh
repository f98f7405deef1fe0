#!/bin/bash
# wgrad_ws1 (size rule) check + in-step A/B, then the torch-glue attribution.
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "wgrad" 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
timeout -k 10 300 python -u tools/ab_inproc.py --switch wgrad_ws1 --blocks 8 --steps 10 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
timeout -k 10 300 python -u tools/torch_prof.py --mode train --steps 3 --rows 80 --stacks > gpurun_out/torch_prof_stdout.txt 2>&1 || exit 1
