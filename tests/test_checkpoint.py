"""Weight conversion: detectron2 -> reference TF
names (restating lib/convert_models/convert_d2.py) -> model parameters.

No detectron2 checkpoint is in the container: the mapping is checked by a
round trip (a model exported to detectron2 names and layouts with the
inverse transforms, converted and loaded into a second model) and by
known answers for the two non-trivial layout rules (box-delta order, fc1 row
order), and since r4 pinned against the reference's own converter
(lib/convert_models/convert_d2.py, pure numpy) by the committed
tests/golden/convert_d2_golden.npz (five layouts, bit-equal arrays).  No
real detectron2 checkpoint is here, so the AP of converted weights is
unmeasured."""
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CATS = {"num_thing_classes": 80, "num_stuff_classes": 53, "stuff_ignore_value": 0}


def _model(seed, yaml="COCO-InstanceSegmentation/mask_rcnn_R_50_FPN_1x.yaml"):
    from detectron2_tensorflow_amd.config import finalize, get_cfg
    from detectron2_tensorflow_amd.modeling import build_model
    cfg = get_cfg()
    cfg.merge_from_file(os.path.join(ROOT, "configs", yaml))
    cfg.MODEL.SEGMENTATION_OUTPUT.FORMAT = "raw"
    finalize(cfg, False, 1, CATS)
    torch.manual_seed(seed)
    m = build_model(cfg)
    with torch.no_grad():
        for _, t in m.reference_variables(include_scope=False):
            t.copy_(torch.rand_like(t) + 0.5)  # distinct, positive (BN variances)
    return cfg, m


def _export_d2(model, cfg):
    """Inverse of convert_weights: our reference-named tensors -> detectron2."""
    from detectron2_tensorflow_amd.checkpoint.convert_d2 import _box_indices
    h = cfg.MODEL.ROI_BOX_HEAD
    res, fc_in = h.POOLER_RESOLUTION, cfg.MODEL.NECK.OUT_CHANNELS
    d = {}
    ren = {"gamma": "norm.weight", "beta": "norm.bias", "moving_mean": "norm.running_mean",
           "moving_variance": "norm.running_var"}
    for name, t in model.reference_variables(include_scope=False):
        if name.endswith("/loss_normalizer"):  # training state: in no detectron2 checkpoint
            continue
        v = t.detach().numpy().copy()
        parts = name.split("/")
        leaf = parts[-1]
        mod = parts[:-2] if parts[-2] == "norm" else parts[:-1]
        path = "/".join(mod)
        if path.startswith("backbone/"):
            p = mod[1:]
            if p[0] == "stem":
                src = "backbone.bottom_up.stem." + p[1]
            else:
                src = f"backbone.bottom_up.{p[0]}.{int(p[1].split('_')[1]) - 1}.{p[2]}"
        elif path.startswith("neck/"):
            src = "backbone." + ".".join(mod[1:])  # (neck/top_block/p6 -> backbone.top_block.p6)
        elif path.startswith("head/head/"):  # the RetinaNet tower (cls_subnet0 -> cls_subnet.0)
            src = "head." + re.sub(r"(subnet)(\d+)$", r"\1.\2", mod[2])
        elif path.startswith("proposal_generator/rpn_head"):
            src = "proposal_generator.rpn_head." + {"share": "conv"}.get(mod[2], mod[2])
        elif path.startswith("roi_heads/box_predictor"):
            src = "roi_heads.box_predictor." + {"class_logits": "cls_score",
                                                "box_deltas": "bbox_pred"}[mod[2]]
        else:
            src = ".".join(mod)
        if leaf in ren:
            d[f"{src}.{ren[leaf]}"] = v
            continue
        is_box = mod[-1] in ("anchor_deltas", "box_deltas", "bbox_pred")
        if leaf == "bias":
            d[src + ".bias"] = v[_box_indices(v.shape[0] // 4)] if is_box else v
            continue
        if v.ndim == 4:  # conv HWIO -> OIHW
            if is_box:
                v = v[..., _box_indices(v.shape[-1] // 4)]
            d[src + ".weight"] = np.ascontiguousarray(v.transpose(3, 2, 0, 1))
        else:  # fc [in, out] -> [out, in]
            if mod[-1] == "fc1":
                v = v.reshape(res, res, fc_in, -1).transpose(2, 0, 1, 3).reshape(res * res * fc_in, -1)
            if is_box:
                v = v[..., _box_indices(v.shape[-1] // 4)]
            d[src + ".weight"] = np.ascontiguousarray(v.T)
    return d


def test_reference_variable_names_follow_the_reference_scopes():
    _, m = _model(0)
    names = [n for n, _ in m.reference_variables(include_scope=False)]
    assert len(names) == len(set(names))
    for want in ("backbone/stem/conv1/weights", "backbone/res2/block_1/shortcut/norm/gamma",
                 "backbone/res4/block_6/conv2/weights", "neck/fpn_lateral2/weights",
                 "neck/fpn_output5/bias", "proposal_generator/rpn_head/share/weights",
                 "roi_heads/box_head/fc1/weights", "roi_heads/box_predictor/box_deltas/weights",
                 "roi_heads/mask_head/mask_fcn4/weights", "roi_heads/mask_head/deconv/weights"):
        assert want in names, want


@pytest.mark.parametrize("yaml", ["COCO-InstanceSegmentation/mask_rcnn_R_50_FPN_1x.yaml",
                                  "COCO-Detection/retinanet_R_50_FPN_1x.yaml"])
def test_detectron2_round_trip_loads_every_variable(yaml):
    """Export -> convert -> strict load.  RetinaNet: its
    loss-normaliser EMA is training state no checkpoint carries -- the strict
    load must not ask for it, and it keeps its initial 100."""
    from detectron2_tensorflow_amd.checkpoint import load_detectron2_checkpoint
    cfg, a = _model(0, yaml)
    _, b = _model(1, yaml)
    d = _export_d2(a, cfg)
    assert len(d) > 300 and "backbone.bottom_up.res2.0.conv1.norm.running_var" in d
    if "retinanet" in yaml:
        assert "head.cls_subnet.0.weight" in d and "backbone.top_block.p6.weight" in d
        with torch.no_grad():
            b.detector.loss_normalizer.fill_(100.0)
    missing, unexpected = load_detectron2_checkpoint(b, d, cfg)
    assert not missing and not unexpected
    for (na, ta), (nb, tb) in zip(a.reference_variables(include_scope=False),
                                  b.reference_variables(include_scope=False)):
        assert na == nb
        if na.endswith("/loss_normalizer"):
            assert float(tb) == 100.0
            continue
        torch.testing.assert_close(tb, ta, rtol=0, atol=0, msg=na)


def test_conversion_kats(tmp_path):
    """Box deltas (dx, dy, dw, dh) -> (dy, dx, dh, dw) per anchor; fc1 row of
    detectron2 input (c, y, x) -> reference row (y * res + x) * C + c; conv
    OIHW -> HWIO; unknown keys are an error; .npz files load without pickle."""
    from detectron2_tensorflow_amd.checkpoint import convert_weights, read_tensor_file
    from detectron2_tensorflow_amd.checkpoint.convert_d2 import _box_indices
    np.testing.assert_array_equal(_box_indices(2), [1, 0, 3, 2, 5, 4, 7, 6])
    cfg, a = _model(0)
    d = _export_d2(a, cfg)
    res, C = 7, 256
    w = np.zeros((1024, C * res * res), np.float32)
    c, y, x = 5, 2, 3
    w[17, c * res * res + y * res + x] = 1.0
    d["roi_heads.box_head.fc1.weight"] = w
    d["proposal_generator.rpn_head.anchor_deltas.bias"] = np.arange(12, dtype=np.float32)
    ow = np.zeros((64, 3, 7, 7), np.float32)
    ow[9, 1, 4, 6] = 2.0
    d["backbone.bottom_up.stem.conv1.weight"] = ow
    out = convert_weights(d, cfg)
    fc1 = out["roi_heads/box_head/fc1/weights"]
    assert fc1[(y * res + x) * C + c, 17] == 1.0 and fc1.sum() == 1.0
    np.testing.assert_array_equal(out["proposal_generator/rpn_head/anchor_deltas/bias"],
                                  [1, 0, 3, 2, 5, 4, 7, 6, 9, 8, 11, 10])
    assert out["backbone/stem/conv1/weights"][4, 6, 1, 9] == 2.0
    with pytest.raises(ValueError):
        convert_weights(dict(d, **{"roi_heads.extra.weight": np.zeros(3)}), cfg)
    p = str(tmp_path / "w.npz")
    np.savez(p, **{"a.b": np.arange(3.0)})
    assert list(read_tensor_file(p)) == ["a.b"]


class _NS:
    def __init__(self, d):
        for k, v in d.items():
            setattr(self, k, _NS(v) if isinstance(v, dict) else v)


def test_convert_weights_matches_reference_fixture():
    """checkpoint.convert_weights against the REFERENCE's own pure-numpy
    convert_d2.convert_weights (lib/convert_models/convert_d2.py:4-187), run
    by tests/golden/make_golden.py on seeded detectron2-named state dicts of
    five layouts (Mask R-CNN R50-FPN, RetinaNet R50 P6P7, C4 Res5ROIHeads with
    class-agnostic boxes, Cascade with a GN conv box head + a deformable
    offset, PanopticFPN): the same reference names, every array equal bit
    for bit (transposes, box-order permutations, fc1 row order)."""
    import json
    from detectron2_tensorflow_amd.checkpoint.convert_d2 import convert_weights
    z = np.load(os.path.join(ROOT, "tests", "golden", "convert_d2_golden.npz"))
    cases = [str(c) for c in z["cases"]]
    assert len(cases) == 5
    for case in cases:
        cfg = _NS(json.loads(str(z[f"{case}|cfg"])))
        pin, pout = f"{case}|in|", f"{case}|out|"
        src = {k[len(pin):]: z[k] for k in z.files if k.startswith(pin)}
        want = {k[len(pout):]: z[k] for k in z.files if k.startswith(pout)}
        got = convert_weights(src, cfg)
        assert sorted(got) == sorted(want), (case, set(got) ^ set(want))
        for k, v in want.items():
            assert got[k].shape == v.shape and np.array_equal(got[k], v), (case, k)
