set -e
for sw in conv_ws_mink=8,16 conv_ws_mink=32,16 wgrad_ws1=3,6 wgrad_ws1=12,6 conv_stream=16384,8192 conv_stream=4096,8192; do
  timeout -k 10 300 python -u tools/ab_inproc.py --switch tune:$sw --blocks 12 --steps 10 > gpurun_out/r5_sweep_${sw%%,*}.log 2>&1
  tail -n 1 gpurun_out/r5_sweep_${sw%%,*}.log
done
