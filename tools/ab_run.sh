set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_geometry.py tests/test_gpu_train.py -x -q -k "roi or grad_share or whole or mask_head or training" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_rb.log 2>&1
tail -2 gpurun_out/t_rb.log
timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 20 > gpurun_out/b_rb.log 2>&1
tail -1 gpurun_out/b_rb.log | python -c "
import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], {k:(v['frac'],v['avg_us'],v['launches']) for k,v in d['kernels'].items() if 'roi' in k})"
