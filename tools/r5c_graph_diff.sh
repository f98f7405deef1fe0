# r5: graphed-vs-eager step diffs after the memset -> fill-kernel change
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/graph_diff.py --steps 7 > gpurun_out/r5c_diff_alt1.log 2>&1 &&
timeout -k 10 300 python -u tools/graph_diff.py --steps 7 > gpurun_out/r5c_diff_alt2.log 2>&1 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 python -u tools/graph_diff.py --steps 7 > gpurun_out/r5c_diff_alt_nopkt.log 2>&1
