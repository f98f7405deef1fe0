# D2MI_CONV_PRIO variants on the kxk + short-K sets (5 = default; 13 = loads at
# priority 1, MFMAs at 2; 21 = activation loads first; 29 = both), twice.
mkdir -p gpurun_out
for rep in 1 2; do for v in 5 13 21 29; do echo "== PRIO=$v"; D2MI_CONV_PRIO=$v timeout -k 10 150 python tools/conv_ab.py --set kxk --iters 30 2>&1 | grep -v amdgpu.ids || exit 1; D2MI_CONV_PRIO=$v timeout -k 10 150 python tools/conv_ab.py --set short_k --iters 30 2>&1 | grep -v amdgpu.ids || exit 1; done; done > gpurun_out/prio2_ab.log 2>&1
