# r6: graph node census (which ops add memset nodes), graphed tests with the
# runtime's packet capture off, then on
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/graph_nodes.py > gpurun_out/r6a_nodes.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_graphed.py > gpurun_out/r6a_graphed_pkt_off.log 2>&1 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_graphed.py -k "not 1333" > gpurun_out/r6a_graphed_pkt_on.log 2>&1
