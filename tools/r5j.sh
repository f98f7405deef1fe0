export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stream_ab.py > gpurun_out/r5j_stream_ab.log 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py -k "stream" > gpurun_out/r5j_stream_test.log 2>&1
