# r6: RetinaNet post, a small level's floor samples spread over the level
# (retina_var 2): parity tests with 12018 forced, then the A/B with stamps on
# the model's head outputs and on iid logits
export TMPDIR=/tmp
mkdir -p gpurun_out
D2MI_RETINA_VAR=12018 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ops.py -k "retinanet_inference" > gpurun_out/r6an_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/retina_post_ab.py --from-model --vars 0,12016,12018 --debug --rounds 7 > gpurun_out/r6an_model.log 2>&1 &&
timeout -k 10 300 python -u tools/retina_post_ab.py --vars 0,12016,12018 --rounds 7 > gpurun_out/r6an_iid.log 2>&1
