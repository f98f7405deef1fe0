set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q -k "fused_1x1 or whole" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_sk.log 2>&1
tail -1 gpurun_out/t_sk.log
bash tools/profile_bench.sh r2c_train --steps 5 --warmup 3 > gpurun_out/pb.log 2>&1
tail -2 gpurun_out/pb.log | cut -c1-250
