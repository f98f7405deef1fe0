set -o pipefail
mkdir -p gpurun_out
T="tests/test_gpu_train.py::test_mask_head_on_foreground_rows_matches_fixed_layout"
timeout -k 10 200 python -u -m pytest $T -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/t1.log 2>&1 || true
D2MI_CONV_OCC=2 timeout -k 10 200 python -u -m pytest $T -x -q --timeout 150 --timeout-method thread -p no:cacheprovider > gpurun_out/t2.log 2>&1 || true
tail -1 gpurun_out/t1.log; tail -1 gpurun_out/t2.log
