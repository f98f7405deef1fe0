#!/bin/bash
# ROIAlign backward pixel-pass ablation (A/B only, results NOT valid for
# arms 3 / 4): tuning roi_bwd_rec 1 = the product pass, 3 = grad_out row index
# folded to 16 rows (row traffic stays in L1/L2: what the row loads cost),
# 4 = runs left in arrival order (what the per-run rank sort costs).
set -eo pipefail
mkdir -p gpurun_out
for arm in 1 3 4; do
  D2MI_ROI_BWD_REC=$arm bash tools/profile_bench.sh abl_$arm --steps 5 --warmup 3
  grep -h "roi_bwd_pixel" gpurun_out/abl_${arm}_timed_kernel_stats.csv | cut -c1-200
done
