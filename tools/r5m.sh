export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_inproc.py --switch tune:conv_stream=1,0 --blocks 10 --steps 10 > gpurun_out/r5m_ab_stream.log 2>&1 &&
timeout -k 10 500 python -u tools/ab_inproc.py --switch tune:roi_bwd_rec=1,0 --blocks 10 --steps 10 > gpurun_out/r5m_ab_roi_rec.log 2>&1
