#!/bin/bash
# ROIAlign backward (counting sort) on the GPU box: the backward parity tests,
# the whole-step training parity tests, the kernel micro-benchmark, the
# in-step kernel timeline, then the conv_epi A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_ops.py -k "roi or crop" 2>&1 | grep -v amdgpu.ids | tail -40 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_train.py tests/test_gpu_layer_api.py 2>&1 | grep -v amdgpu.ids | tail -5 || exit 1
timeout -k 10 200 python -u tools/bench_kernels.py --only roi 2>&1 | grep -v amdgpu.ids || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_roibwd -o run -- \
  python bench.py --steps 5 --warmup 3 > gpurun_out/prof_roibwd.log 2>&1 || exit 1
python tools/roi_bwd_timeline.py gpurun_out/prof_roibwd 2>&1 | tail -30
bash tools/epi_ab.sh
