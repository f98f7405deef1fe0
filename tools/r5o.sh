#!/bin/bash
# r5: fused RetinaNet post-processing -- parity (12 cases), A/B vs the unfused
# pipeline, kernel stats of the fused path; stream 1x1 parity with the widened
# shape set
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py -x -v --timeout 120 --timeout-method thread -k "retinanet_inference or conv1x1_stream" > gpurun_out/r5o_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/retina_post_ab.py > gpurun_out/r5o_ab.log 2>&1 &&
timeout -k 10 200 python -u tools/retina_post_ab.py --dist saturated --iters 3 --rounds 2 > gpurun_out/r5o_ab_saturated.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r5o_prof -o run -- python3 tools/retina_post_ab.py --arms 1 --iters 10 --rounds 2 > gpurun_out/r5o_prof.log 2>&1
