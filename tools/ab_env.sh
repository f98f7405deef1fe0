# Training-bench A/B of environment knobs (run on the box), plus host time.
# usage: tools/ab_env.sh "VAR=a VAR2=b" "VAR=c" ...   (one bench per setting, twice)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_time.py --steps 5 > gpurun_out/host_time.log 2>&1 && tail -3 gpurun_out/host_time.log
for rep in 1 2; do
for setting in "$@"; do
  env $setting timeout -k 10 200 python bench.py --steps 20 --cpu-baseline 0 > gpurun_out/ab_env.log 2>&1 || exit 1
  python -c "import json,sys;d=json.loads(open('gpurun_out/ab_env.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['frac'])" "$setting"
done
done
