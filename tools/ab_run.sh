set -o pipefail
mkdir -p gpurun_out
o=gpurun_out/ab4.log
: > $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv" --timeout 120 --timeout-method thread -p no:cacheprovider >> $o 2>&1
for occ in 2 3; do
echo "occ=$occ" >> $o
D2MI_CONV_OCC=$occ timeout -k 10 120 python tools/conv_ab.py --set short_k >> $o 2>&1
D2MI_CONV_OCC=$occ timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 20 >> $o 2>&1
done
D2MI_CONV_OCC=2 timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 20 >> $o 2>&1
timeout -k 10 200 python bench.py --cpu-baseline 0 --steps 20 >> $o 2>&1
cat $o | grep -v amdgpu.ids | cut -c1-400
