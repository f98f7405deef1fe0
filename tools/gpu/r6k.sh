# r6: do replayed graphs run forked branches concurrently (packet capture on /
# off)?  then the ROIAlign ceilings (cold and maps-rewritten)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/graph_parallel_probe.py > gpurun_out/r6k_graph_parallel.log 2>&1 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 python -u tools/graph_parallel_probe.py >> gpurun_out/r6k_graph_parallel.log 2>&1 &&
timeout -k 10 400 python -u tools/gather_ceiling.py --iters 20 --rounds 5 > gpurun_out/r6i_gather_ceiling.log 2>&1
