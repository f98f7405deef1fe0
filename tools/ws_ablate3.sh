# WS conv ablations (D2MI_CONV_DBG bits: 1 no loads, 2 no LDS staging, 4 no MFMA
# loop, 8 no epilogue; r3 also had 16 / 32 = no B / A split VALU, since removed:
# profiles/r3b_ws_ablate3.log)
set -o pipefail
mkdir -p gpurun_out
S="2,200,336,256,256,3,1,plain;2,50,84,256,256,3,1,plain;2,50,84,1024,256,1,1,plain;2,100,168,128,128,3,1,plain"
for v in 0 16 32 48 2 1 3 4 ${EXTRA}; do echo "== DBG=$v"; D2MI_CONV_DBG=$v timeout -k 10 120 python tools/conv_ab.py --shapes "$S" 2>&1 | grep -v amdgpu.ids || exit 1; done > gpurun_out/ws_ablate3.log 2>&1
cat gpurun_out/ws_ablate3.log
