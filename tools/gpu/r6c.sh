# r6: graph-replayed data parallelism -- the DP tests (eager / graphed over
# gloo, the RCCL world-1 child with a graphed arm) and the 2-rank bench rehearsal
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_dp.py > gpurun_out/r6c_dp_tests.log 2>&1 &&
bash tools/dp_rehearse.sh r6c_dp_rehearse
