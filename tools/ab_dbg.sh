# Conv ablations (D2MI_CONV_DBG bits: 1 no loads, 2 no LDS staging, 4 no MFMA loop, 8 no epilogue)
set -o pipefail
mkdir -p gpurun_out
S="2,200,336,256,256,3,1,plain;2,50,84,256,256,3,1,plain;2,50,84,256,1024,1,1,r"
for v in 0 1 2 3 4 5 6 8 11 12 ${EXTRA}; do echo "== DBG=$v"; D2MI_CONV_DBG=$v timeout -k 10 120 python tools/conv_ab.py --shapes "$S" 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/dbg_ab.log 2>&1
cat gpurun_out/dbg_ab.log
