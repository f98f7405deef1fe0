#!/bin/bash
# ROIAlign backward pixel-pass ablation (A/B only, results NOT valid for
# arms 3..6): tuning roi_bwd_rec 1 = the product pass, 3 = grad_out row index
# folded to 16 rows (row traffic stays in L1/L2: what the row loads cost),
# 4 = runs left in arrival order (what the per-run rank sort costs),
# 5 / 6 = at most 8 / 24 contributions summed per run (what the long runs'
# dependent row batches cost).  Then the product pass's per-call durations,
# grid and register counts from one kernel trace.
set -eo pipefail
mkdir -p gpurun_out
for arm in ${ARMS-1 3 4}; do
  D2MI_ROI_BWD_REC=$arm bash tools/profile_bench.sh abl_$arm --steps 5 --warmup 3
  grep -h "roi_bwd_pixel" gpurun_out/abl_${arm}_timed_kernel_stats.csv | cut -c1-200
done
export TMPDIR=/tmp
rm -rf gpurun_out/prof_roi_calls
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_roi_calls -o run \
    -- python3 bench.py --cpu-baseline 0 --no-kernel-timing --steps 2 --warmup 2 > gpurun_out/prof_roi_calls.log 2>&1
python3 - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/prof_roi_calls/**/*kernel_trace.csv", recursive=True))[0]
rows = [r for r in csv.DictReader(open(f)) if "roi_bwd" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
with open("gpurun_out/r5_roi_bwd_calls.txt", "w") as out:
    for r in rows[-40:]:
        n = r["Kernel_Name"].replace("void ", "").replace("d2mi::(anonymous namespace)::", "").split("(")[0]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
        out.write(f"{n[:48]:48s} {d:8.1f} us grid {grid:>9s} "
                  f"vgpr {r.get('Arch_VGPR_Count', r.get('VGPR_Count', '?'))} lds {r.get('LDS_Block_Size', r.get('Lds_Size', '?'))}\n")
    out.write("columns: " + ",".join(rows[0].keys()) + "\n")
print(open("gpurun_out/r5_roi_bwd_calls.txt").read())
PY
find gpurun_out/prof_roi_calls -name "*trace.csv" -delete
