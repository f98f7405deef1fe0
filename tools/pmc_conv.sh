#!/bin/bash
# SQ / LDS PMC counters of one conv shape (tools/conv_one.py) per math mode.
# usage: tools/pmc_conv.sh "<N,H,W,Cin,Cout,k,s>" mode...
set -o pipefail
export TMPDIR=/tmp
shape=$1; shift
mkdir -p gpurun_out/pmc_conv
for mode in "$@"; do
timeout -k 10 120 python -u tools/conv_one.py --shape $shape --mode $mode --iters 10 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d gpurun_out/pmc_conv/$mode -o run -- python3 tools/conv_one.py --shape $shape --mode $mode --iters 3 > gpurun_out/pmc_conv/$mode.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_conv/${mode}_b -o run -- python3 tools/conv_one.py --shape $shape --mode $mode --iters 3 > gpurun_out/pmc_conv/${mode}_b.log 2>&1 || exit 3
done
