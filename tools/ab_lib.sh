# A/B of two builds of libd2mi_hip.so (D2MI_LIB) on conv_ab.py shape sets,
# alternating A B A B; the printed output sums must agree (same arithmetic).
# usage: tools/ab_lib.sh <lib A> <lib B> [sets, default "kxk short_k"]
mkdir -p gpurun_out
A=$1; B=$2; sets=${3:-"kxk short_k"}
for rep in 1 2; do for lib in $A $B; do echo "== LIB=$(basename $lib)"; for st in $sets; do
  D2MI_LIB=$lib timeout -k 10 150 python tools/conv_ab.py --set $st --iters 30 2>&1 | grep -v amdgpu.ids || exit 1
done; done; done > gpurun_out/lib_ab.log 2>&1
