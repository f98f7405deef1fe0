# r6: the aten ops of one eager training step by Python call site (torch
# glue between the d2mi kernels)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/glue_sites.py --rows 80 > gpurun_out/r6ak_glue_sites.log 2>&1
