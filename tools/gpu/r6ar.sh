# r6: which torch kernels an eager training step still launches, and from
# where (tools/torch_op_census.py: torch.profiler, stacks, device time)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/torch_op_census.py > gpurun_out/${CENSUS_OUT:-r6ar_torch_op_census.txt} 2>&1
