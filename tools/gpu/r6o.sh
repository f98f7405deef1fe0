# r6: the Mask R-CNN 1333x800 stage-wise test
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_gpu_model.py -k "mask_rcnn_1333x800" > gpurun_out/r6o_mask_1333.log 2>&1
