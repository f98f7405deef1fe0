# r6: graphed tests with the runtime's graph packet capture ON (its default)
# now that no capture holds a memset node; then the training bench with
# packet capture on / off, alternating on one box
export TMPDIR=/tmp
mkdir -p gpurun_out
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_graphed.py > gpurun_out/r6b_graphed_pkt_on.log 2>&1 &&
for i in 1 2; do
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 20 > gpurun_out/r6b_bench_pkt_on_$i.log 2>&1 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python -u bench.py --cpu-baseline 0 --fixed-rows-steps 0 --steps 20 > gpurun_out/r6b_bench_pkt_off_$i.log 2>&1 || exit 1
done
