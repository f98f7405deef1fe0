# r6: DP tests + rehearsal, the tests touched by the r6 ADVICE fixes, and the
# int8-MFMA Matrix NMS (SOLO tail tests, both paths; the C5 bench line each way)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_solo.py -k "tail" > gpurun_out/r6d_solo.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_dp.py > gpurun_out/r6d_dp_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py tests/test_gpu_ops.py -k "sgd or topk or rpn_proposals or stream_kernel" > gpurun_out/r6d_ops.log 2>&1 &&
D2MI_SOLO_MFMA=1 timeout -k 10 300 python -u bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 > gpurun_out/r6d_solo_bench_mfma.log 2>&1 &&
D2MI_SOLO_MFMA=0 timeout -k 10 300 python -u bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 > gpurun_out/r6d_solo_bench_popcount.log 2>&1 &&
bash tools/dp_rehearse.sh r6d_dp_rehearse
