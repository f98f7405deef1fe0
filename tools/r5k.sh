export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stream_ab.py > gpurun_out/r5k_stream_ab.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train.py -k "stream or roi or deferred or whole_training" > gpurun_out/r5k_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 > gpurun_out/r5k_bench.log 2>&1
