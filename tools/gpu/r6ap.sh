# r6: RetinaNet collect with ordinary loads (retina_var 16384) on the model's
# head outputs (fresh logits: written by the head just before) and on iid logits
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/retina_post_ab.py --from-model --vars 12018,28402 --rounds 7 > gpurun_out/r6ap_model.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 12018,28402 --rounds 7 > gpurun_out/r6ap_iid.log 2>&1
