# r5: stream 1x1 conv per-shape A/B, parity tests, in-step A/Bs (ROI backward run records, stream conv), bench
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stream_ab.py > gpurun_out/r5l_stream_ab.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_train.py -k "stream or roi or deferred or whole_training" > gpurun_out/r5l_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_inproc.py --switch tune:roi_bwd_rec=1,0 --blocks 6 --steps 10 > gpurun_out/r5l_ab_roi_rec.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_inproc.py --switch tune:conv_stream=1,0 --blocks 6 --steps 10 > gpurun_out/r5l_ab_stream.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/r5l_bench.log 2>&1
