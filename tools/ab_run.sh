set -o pipefail
mkdir -p gpurun_out
o=gpurun_out/ab_ppw.log; : > $o
D2MI_ROI_BWD_PPW=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "grad_share or backward" --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -1 >> $o
for v in 4 8 4 8; do
D2MI_ROI_BWD_PPW=$v timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 20 2>&1 | tail -1 | python -c "
import sys,json; d=json.loads(sys.stdin.read()); print('$v', d['value'], {k:(v['frac'],v['avg_us']) for k,v in d['kernels'].items() if 'roi_align_bwd' in k})" >> $o
done
cat $o
