# r6: PMC of the int8-MFMA intersection kernel (SQ pass, separate from any trace)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "solo_inter_mfma" -d gpurun_out/pmc_r6g_sq -o sq -- python bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 --steps 2 --warmup 1 --no-calibration > gpurun_out/r6g_pmc_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-include-regex "solo_inter_mfma" -d gpurun_out/pmc_r6g_sq2 -o sq2 -- python bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 --steps 2 --warmup 1 --no-calibration > gpurun_out/r6g_pmc_sq2.log 2>&1
