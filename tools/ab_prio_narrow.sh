# D2MI_CONV_PRIO 1 vs 5 (bit 4: priority in the double-buffered narrow-Cout
# kernels' MFMA phase) on the narrow shapes, then the training bench.
mkdir -p gpurun_out
S="2,200,336,256,64,1,1,plain;2,200,336,64,64,3,1,plain;2,200,336,64,64,1,1,plain;2,100,168,256,64,1,1,plain;32,14,14,256,64,1,1,plain;2,200,336,256,16,1,1,plain"
for v in 1 5 1 5; do echo "== PRIO=$v"; D2MI_CONV_PRIO=$v timeout -k 10 150 python tools/conv_ab.py --shapes "$S" --iters 30 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/prio_narrow.log 2>&1
for v in 1 5 1 5; do D2MI_CONV_PRIO=$v timeout -k 10 200 python bench.py --steps 20 --cpu-baseline 0 > gpurun_out/prio_b.log 2>&1 || exit 2; python -c "import json,sys;d=json.loads(open('gpurun_out/prio_b.log').read().strip().splitlines()[-1]);print('PRIO', sys.argv[1], d['value'], d['ms_per_step'])" $v; done
