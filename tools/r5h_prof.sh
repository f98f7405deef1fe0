# r5: per-shape conv roofline classification + kernel-trace profile of the graphed bench step
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/conv_shapes.py --steps 3 > gpurun_out/r5h_conv_shapes.txt 2>&1 &&
STEPS=5 bash tools/profile_bench.sh r5h_graphs --steps 5 --warmup 3 --fixed-rows-steps 0
