set -e
for sw in conv_ws_mintiles=50,0 conv_ws_mintiles=100,0 conv_ws_mintiles=200,0; do
  timeout -k 10 300 python -u tools/ab_inproc.py --switch tune:$sw --blocks 12 --steps 10 > gpurun_out/r5_sweep_${sw%%,*}.log 2>&1
  tail -n 1 gpurun_out/r5_sweep_${sw%%,*}.log
done
