"""Generates tests/golden/nms_golden.npz from the REFERENCE's own numpy NMS.

Runs only in the build container (needs /root/reference): loads
lib/structures/np_box_list.py, np_box_ops.py and np_box_list_ops.py by file
path under a synthetic package (bypassing lib/structures/__init__.py, which
imports TensorFlow) and records, for seeded inputs, the indices kept by
np_box_list_ops.non_max_suppression (np_box_list_ops.py:146-217).

That numpy NMS matches TF's NonMaxSuppressionV3 only on inputs that avoid its
documented differences (float64 intersection, no min/max corner normalisation,
no area<=0 rule, argsort tie order), so the generator draws positive-area,
tie-free inputs and rejects sets with any pairwise IoU within 1e-4 of the
threshold.  The committed .npz is data (inputs + expected outputs); no
reference source travels with it.

    python tests/golden/make_golden.py [/root/reference]
"""
import importlib.util
import os
import sys
import types

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "nms_golden.npz")


def load_reference_np_ops(ref_root):
    sdir = os.path.join(ref_root, "lib", "structures")
    pkg = types.ModuleType("_refstruct")
    pkg.__path__ = [sdir]
    sys.modules["_refstruct"] = pkg
    mods = {}
    for name in ["np_box_list", "np_box_ops", "np_box_list_ops"]:
        spec = importlib.util.spec_from_file_location(f"_refstruct.{name}",
                                                      os.path.join(sdir, name + ".py"))
        m = importlib.util.module_from_spec(spec)
        sys.modules[f"_refstruct.{name}"] = m
        spec.loader.exec_module(m)
        setattr(pkg, name, m)
        mods[name] = m
    return mods


def random_boxes(rng, n, extent=800.0, min_side=4.0, max_side=200.0, clusters=None):
    if clusters:
        centers = rng.uniform(0, extent, size=(clusters, 2))
        c = centers[rng.integers(0, clusters, size=n)] + rng.normal(0, 12, size=(n, 2))
    else:
        c = rng.uniform(0, extent, size=(n, 2))
    hw = np.exp(rng.uniform(np.log(min_side), np.log(max_side), size=(n, 2)))
    b = np.concatenate([c - hw / 2, c + hw / 2], axis=1)
    return b.astype(np.float32)


def iou64(b):
    b = b.astype(np.float64)
    a = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    ih = np.clip(np.minimum(b[:, None, 2], b[None, :, 2]) - np.maximum(b[:, None, 0], b[None, :, 0]), 0, None)
    iw = np.clip(np.minimum(b[:, None, 3], b[None, :, 3]) - np.maximum(b[:, None, 1], b[None, :, 1]), 0, None)
    inter = ih * iw
    return inter / (a[:, None] + a[None, :] - inter)


def make_case(rng, mods, n, thr, max_out, clusters):
    for _ in range(100):
        boxes = random_boxes(rng, n, clusters=clusters)
        iou = iou64(boxes)
        np.fill_diagonal(iou, 0)
        if np.any(np.abs(iou - thr) < 1e-4):
            continue
        scores = rng.permutation(n).astype(np.float32) / np.float32(n) + np.float32(0.001)
        bl = mods["np_box_list"].BoxList(boxes.copy())
        bl.add_field("scores", scores.copy())
        bl.add_field("idx", np.arange(n))
        res = mods["np_box_list_ops"].non_max_suppression(bl, max_output_size=max_out,
                                                          iou_threshold=thr,
                                                          score_threshold=-np.inf)
        keep = res.get_field("idx").astype(np.int32)
        return boxes, scores, keep
    raise RuntimeError("could not draw a threshold-safe case")


def main(ref_root="/root/reference"):
    mods = load_reference_np_ops(ref_root)
    rng = np.random.default_rng(20261015)
    cases = [
        (64, 0.5, 64, None), (64, 0.3, 10, 4), (300, 0.7, 1000, 20), (1000, 0.7, 1000, 60),
        (1000, 0.5, 100, 30), (2000, 0.7, 1000, 100), (2000, 0.5, 300, 40), (5, 0.5, 5, None),
    ]
    data = {}
    for i, (n, thr, max_out, clusters) in enumerate(cases):
        b, s, k = make_case(rng, mods, n, thr, max_out, clusters)
        data[f"c{i}_boxes"] = b
        data[f"c{i}_scores"] = s
        data[f"c{i}_keep"] = k
        data[f"c{i}_params"] = np.array([thr, max_out], np.float64)
    data["num_cases"] = np.array(len(cases))
    np.savez_compressed(OUT, **data)
    print("wrote", OUT, {k: v.shape for k, v in data.items() if k.endswith("_keep")})


if __name__ == "__main__":
    main(*sys.argv[1:])
