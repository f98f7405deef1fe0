# r6: stamps inside the RetinaNet NMS's first tile (rows, barrier, resolve)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,1744 --debug --rounds 3 > gpurun_out/r6y_ab.log 2>&1
