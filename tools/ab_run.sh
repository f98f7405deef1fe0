set -o pipefail
mkdir -p gpurun_out
o=gpurun_out/ab_w.log; : > $o
for occ in 2 3; do
echo "wocc=$occ" >> $o
D2MI_WGRAD_OCC=$occ timeout -k 10 120 python tools/conv_ab.py --set wgrad --iters 20 2>&1 | grep -v amdgpu >> $o
D2MI_WGRAD_OCC=$occ timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 20 2>&1 | tail -1 | cut -c1-100 >> $o
done
D2MI_WGRAD_OCC=2 timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 20 2>&1 | tail -1 | cut -c1-100 >> $o
timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 20 2>&1 | tail -1 | cut -c1-100 >> $o
cat $o
