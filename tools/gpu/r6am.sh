# r6: RetinaNet post without the windowed rank (11984) vs with the rank
# launch's rounds capped and looped (12016), on the model's own head outputs
# and on iid logits; parity tests with 12016 forced first
export TMPDIR=/tmp
mkdir -p gpurun_out
D2MI_RETINA_VAR=12016 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "retinanet_inference" > gpurun_out/r6am_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/retina_post_ab.py --from-model --vars 0,11984,12016,16080 --rounds 7 > gpurun_out/r6am_model.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,11984,12016,16080 --rounds 7 > gpurun_out/r6am_iid.log 2>&1
