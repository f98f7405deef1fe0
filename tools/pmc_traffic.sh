#!/bin/bash
# HBM traffic per launch of the hot kernels from rocprofv3 PMC counters (run on
# the GPU box).  Two separate passes (FETCH_SIZE and WRITE_SIZE cannot share a
# pass on gfx950), each with --kernel-trace only, as MI355X_MICROARCH.md's
# HBM/rocprofv3 section prescribes; tools/pmc_summarize.py applies its gfx950
# correction (FETCH_SIZE counts half the bytes of 16 B/lane reads).
# usage: tools/pmc_traffic.sh <tag> [bench args...]
set -eo pipefail
tag=$1; shift
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  out=gpurun_out/pmc_${tag}_$c
  rm -rf "$out"
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$out" -o run \
      -- python3 bench.py --cpu-baseline 0 --no-kernel-timing "$@" > "$out.log" 2>&1
done
python3 tools/pmc_summarize.py gpurun_out/pmc_${tag}_FETCH_SIZE gpurun_out/pmc_${tag}_WRITE_SIZE \
    gpurun_out/${tag}_pmc.json
find gpurun_out/pmc_${tag}_* -name "*.csv" -size +20M -delete
