# Wave-priority A/B: conv (D2MI_CONV_PRIO 0 / 1 / 2, default 1) on the kxk and
# short-K sets, the split wgrad (D2MI_WGRAD_PRIO 0 / 1) on the wgrad set, then
# the training bench alternating the settings.
mkdir -p gpurun_out
for v in 0 1 2; do echo "== PRIO=$v"; D2MI_CONV_PRIO=$v timeout -k 10 150 python tools/conv_ab.py --set kxk --iters 30 2>&1 | grep -v amdgpu.ids || exit 1; D2MI_CONV_PRIO=$v timeout -k 10 150 python tools/conv_ab.py --set short_k --iters 30 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/prio_ab.log 2>&1
for v in 0 1; do echo "== WPRIO=$v"; D2MI_WGRAD_PRIO=$v timeout -k 10 150 python tools/conv_ab.py --set wgrad --iters 30 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/wprio_ab.log 2>&1
for v in ${BENCH_SETTINGS:-"D2MI_CONV_PRIO=0" "D2MI_CONV_PRIO=1" "D2MI_CONV_PRIO=0" "D2MI_CONV_PRIO=1"}; do env $v timeout -k 10 200 python bench.py --steps 20 --cpu-baseline 0 > gpurun_out/prio_b.log 2>&1 || exit 2; python -c "import json,sys;d=json.loads(open('gpurun_out/prio_b.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['frac'], d['kernels']['conv2d_wgrad_split']['frac'])" $v; done
