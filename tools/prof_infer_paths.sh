set -o pipefail
bash tools/profile_bench.sh r2x_solo --model solo_v2_R_50_FPN --mode infer --steps 5 --warmup 3 > /dev/null
bash tools/profile_bench.sh r2x_infer --mode infer --steps 5 --warmup 3 > /dev/null
for t in solo infer; do echo "== $t"; python3 - $t <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f'gpurun_out/r2x_{sys.argv[1]}_timed_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/5/1000:.1f} us/step")
for r in rows[:40]:
    print(f"{int(r['Calls'])/5:6.1f}/step {float(r['TotalDurationNs'])/5000:8.1f} us  {r['Name'][:90]}")
PY
done
