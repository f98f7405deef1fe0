# r6: RetinaNet post on the calibrated model's own head outputs (the in-model
# score distribution): phase stamps; 11984 = no windowed rank, 10960 = also
# no fast IoU, 8912 = also no fixed-point resolve
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/retina_post_ab.py --from-model --vars 0,16080,11984,10960,8912 --debug --rounds 5 > gpurun_out/r6al_ab.log 2>&1
