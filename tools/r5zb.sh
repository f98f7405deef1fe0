#!/bin/bash
# r5: RPN merge rank + signed-zero key canonicalisation -- full GPU suite,
# then the in-step A/B of rpn_merge
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r5zb_tests.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_inproc.py --switch tune:rpn_merge=1,0 --blocks 10 --steps 10 > gpurun_out/r5zb_ab_merge.log 2>&1
