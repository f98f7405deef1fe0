set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4o_smoke.log 2>&1 || { tail -20 gpurun_out/r4o_smoke.log; exit 1; }
tail -1 gpurun_out/r4o_smoke.log
timeout -k 10 500 python3 bench.py > gpurun_out/r4o_bench.log 2>&1 || { tail -20 gpurun_out/r4o_bench.log; exit 1; }
tail -1 gpurun_out/r4o_bench.log | cut -c1-400
