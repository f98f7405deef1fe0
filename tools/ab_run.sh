set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_retinanet.py tests/test_solo.py -x -q -k "levels or retinanet or solo" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_lv.log 2>&1
tail -2 gpurun_out/t_lv.log
timeout -k 10 300 python bench.py --model retinanet_R_101_FPN --mode infer --cpu-baseline 0 > gpurun_out/b_ret.log 2>&1
tail -1 gpurun_out/b_ret.log | cut -c1-300
timeout -k 10 300 python bench.py --model solo_v2_R_50_FPN --mode infer --cpu-baseline 0 > gpurun_out/b_solo.log 2>&1
tail -1 gpurun_out/b_solo.log | cut -c1-300
