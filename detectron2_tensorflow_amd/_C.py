"""ctypes binding of libd2mi_hip.so (the C ABI declared in include/d2mi.h).

The library is built in-tree (``detectron2_tensorflow_amd/_build.py``) and is
the only compute path of the hot ops: if it cannot be loaded, every op raises
(there is no CPU or eager fallback).  torch is imported first so that the HIP
runtime torch ships (``libamdhip64.so.7``) is the one the library binds to;
device pointers and ``hipStream_t`` handles are passed straight from torch.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# D2MI_LIB: an alternative build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get("D2MI_LIB") or os.path.join(_HERE, "lib", "libd2mi_hip.so")

_lib = None
_load_error = None

c_int, c_float, c_size_t, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p
c_char_p = ctypes.c_char_p
P = c_void_p  # device or host pointer

# name -> (restype, argtypes)
_SIGS = {
    "d2mi_version": (c_int, []),
    "d2mi_source_hash": (c_char_p, []),
    "d2mi_set_tuning": (c_int, [c_char_p, c_int]),
    "d2mi_get_tuning": (c_int, [c_char_p]),
    "d2mi_last_error": (c_char_p, []),
    "d2mi_error_word_dev": (c_void_p, []),
    "d2mi_clear_errors": (c_int, [P]),
    "d2mi_graph_census": (c_int, [P, P, c_int]),
    "d2mi_capture_census": (c_int, [P, P, c_int]),
    "d2mi_roi_align_fwd": (c_int, [P, P, P, c_int, c_int, P, P, c_int, c_int, c_int, c_int, c_int,
                                   c_int, c_int, c_int, c_int, c_int, c_int, P, P, P]),
    "d2mi_roi_align_bwd_workspace_size": (c_size_t, [P, c_int, c_int, c_int, c_int, c_int, c_int]),
    "d2mi_roi_align_bwd": (c_int, [P, P, P, c_int, c_int, P, P, c_int, c_int, c_int, c_int, c_int,
                                   c_int, c_int, c_int, c_int, c_int, c_int, P, P, c_size_t, P]),
    "d2mi_roi_align_bwd_ex": (c_int, [P, P, P, c_int, c_int, P, P, c_int, c_int, c_int, c_int,
                                      c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, c_int,
                                      P, c_size_t, P]),
    "d2mi_roi_align_bwd2_workspace_size": (c_size_t, [P, c_int, c_int, c_int, c_int, c_int, c_int,
                                                   c_int, c_int, c_int, c_int]),
    "d2mi_roi_align_bwd2": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_int, c_int, P, P, c_int, c_int, c_int, c_int, P, P, P, c_int,
                                    c_int, c_int, c_int, P, c_int, P, c_size_t, P]),
    "d2mi_roi_align_bwd2_ex": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                       c_int, c_int, P, P, c_int, c_int, c_int, c_int, P, P, P,
                                       c_int, c_int, c_int, c_int, P, c_int, c_int, c_int, c_int,
                                       P, c_size_t, P]),
    "d2mi_nms_workspace_size": (c_size_t, [c_int, c_int]),
    "d2mi_nms": (c_int, [P, P, P, c_int, c_int, c_int, c_float, P, P, P, c_size_t, P]),
    "d2mi_topk_workspace_size": (c_size_t, [c_int, c_int]),
    "d2mi_topk": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, P, P, P, c_size_t, P]),
    "d2mi_subsample_workspace_size": (c_size_t, [c_int, c_int]),
    "d2mi_subsample": (c_int, [P, c_int, c_int, ctypes.c_longlong, c_int, c_int, P, P, P, P, P,
                               c_int, P, c_size_t, P]),
    "d2mi_grid_anchors": (c_int, [c_int, c_int, c_float, P, c_int, P, P]),
    "d2mi_apply_deltas": (c_int, [P, P, c_int, c_int, P, c_float, P, P]),
    "d2mi_rpn_proposals_workspace_size": (c_size_t, [c_int, c_int, P, c_int, c_int, c_int]),
    "d2mi_rpn_proposals": (c_int, [P, P, P, P, P, c_int, c_int, c_int, P, c_int, c_int, c_float,
                                   c_float, P, c_float, P, P, P, P, c_size_t, P]),
    "d2mi_rpn_proposals_ex": (c_int, [P, P, P, P, P, P, P, c_int, c_int, c_int, P, c_int, c_int,
                                      c_float, c_float, P, c_float, P, P, P, P, c_size_t, P]),
    "d2mi_rpn_head_gather": (c_int, [P, P, c_int, c_int, c_int, c_int, P, P, P]),
    "d2mi_rpn_head_scatter": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, P]),
    "d2mi_fast_rcnn_workspace_size": (c_size_t, [c_int, c_int, c_int, c_float, c_int]),
    "d2mi_fast_rcnn_inference": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, P, P,
                                         c_float, c_float, c_float, c_int, P, P, P, P, P, P,
                                         c_size_t, P]),
    "d2mi_retinanet_workspace_size": (c_size_t, [c_int, c_int, P, c_int, c_int, c_int]),
    "d2mi_retinanet_inference": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_float,
                                         c_float, c_int, P, c_float, P, P, P, P, P, c_size_t, P]),
    "d2mi_matrix_nms_workspace_size": (c_size_t, [c_int]),
    "d2mi_matrix_nms": (c_int, [P, P, P, P, c_int, c_int, c_int, c_float, P, P, c_size_t, P]),
    "d2mi_resize_bilinear": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P,
                                     P]),
    "d2mi_solo_cells": (c_int, [P, P, c_int, c_int, c_int, c_float, P, P, P, P, P]),
    "d2mi_solo_mask_stats": (c_int, [P, c_int, c_int, c_float, P, P, P]),
    "d2mi_solo_select_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int]),
    "d2mi_solo_select": (c_int, [P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_float,
                                 c_float, c_int, P, P, P, P, P, P, c_size_t, P]),
    "d2mi_solo_matrix_nms_workspace_size": (c_size_t, [c_int, c_int]),
    "d2mi_solo_matrix_nms": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_float, P, P,
                                     c_size_t, P]),
    "d2mi_solo_finalize_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "d2mi_solo_finalize": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_float, c_int,
                                   c_float, c_int, c_int, P, P, P, P, P, P, c_size_t, P]),
    "d2mi_group_norm_workspace_size": (c_size_t, [c_int] * 5),
    "d2mi_group_norm_nhwc": (c_int, [P, c_int, c_int, c_int, c_int, c_int, P, P, c_float, c_int,
                                     c_int, c_int, P, P, c_size_t, P]),
    "d2mi_group_norm_levels_workspace_size": (c_size_t, [P, c_int, c_int, c_int]),
    "d2mi_group_norm_nhwc_levels": (c_int, [P, P, c_int, c_int, c_int, P, P, c_float, c_int, P, P,
                                            c_size_t, P]),
    "d2mi_conv_pack_weights": (c_int, [P, c_int, c_int, c_int, c_int, P, P]),
    "d2mi_conv_pack_weights_many": (c_int, [c_int, P, P, P, P]),
    "d2mi_conv2d_nhwc": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                                 c_int, c_int, c_int, c_int, c_int, P]),
    "d2mi_conv2d_workspace_size": (c_size_t, [c_int] * 10),
    "d2mi_conv2d_wgrad_workspace_size": (c_size_t, [c_int] * 10),
    "d2mi_fold_frozen_bn": (c_int, [P, P, P, P, P, P, c_float, c_int, c_int, c_int, c_int, P, P,
                                    P, P]),
    "d2mi_fold_frozen_bn_bwd_workspace_size": (c_size_t, [c_int]),
    "d2mi_fold_frozen_bn_bwd": (c_int, [P, P, P, P, P, P, P, c_float, c_int, c_int, c_int, c_int,
                                        P, P, P, P, P, c_size_t, P]),
    "d2mi_conv2d_wgrad": (c_int, [P, P, P, P] + [c_int] * 10 + [P, c_size_t, P]),
    "d2mi_conv2d_wgrad_ex": (c_int, [P, P, P, P] + [c_int] * 11 + [P, c_size_t, P]),
    "d2mi_conv2d_nhwc_ex": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_int, c_int, c_int, c_int, c_int, P, c_size_t, P]),
    "d2mi_conv2d_nhwc_gated": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_int,
                                       c_int, c_int, c_int, c_int, c_int, c_int, P, c_size_t, P]),
    "d2mi_conv2d_levels_workspace_size": (c_size_t, [P, c_int, c_int, c_int, c_int, c_int, c_int,
                                                  c_int, c_int]),
    "d2mi_conv2d_nhwc_levels": (c_int, [P, P, c_int, P, P, P, c_int, c_int, c_int, c_int, c_int,
                                        c_int, c_int, c_int, P, c_size_t, P]),
    "d2mi_split_bf16x3": (c_int, [P, ctypes.c_int64, P, P]),
    "d2mi_paste_masks": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, c_float, P, P]),
    "d2mi_wgrad_skinny_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "d2mi_wgrad_skinny": (c_int, [P, P, c_int, c_int, c_int, P, P, P, c_size_t, P]),
    "d2mi_wgrad_skinny_ex": (c_int, [P, P, c_int, c_int, c_int, P, P, c_int, P, c_size_t, P]),
    "d2mi_wgrad_skinny_levels_workspace_size": (c_size_t, [P, c_int, c_int, c_int]),
    "d2mi_wgrad_skinny_levels": (c_int, [P, P, P, c_int, c_int, c_int, P, P, c_int, P, c_size_t,
                                         P]),
    "d2mi_column_sum_workspace_size": (c_size_t, [ctypes.c_longlong, c_int]),
    "d2mi_column_sum": (c_int, [P, ctypes.c_longlong, c_int, P, P, c_size_t, P]),
    "d2mi_upsample2x_grad": (c_int, [P, c_int, c_int, c_int, c_int, P, P]),
    "d2mi_stride_scatter": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "d2mi_stride_scatter_ex": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "d2mi_match_workspace_size": (c_size_t, [c_int, c_int]),
    "d2mi_match_boxes": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, P, c_int, c_int, c_float,
                                 c_float, P, P, P, c_size_t, P]),
    "d2mi_match_boxes_ex": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, P, P, c_int, c_int,
                                    c_float, c_float, P, P, P, c_size_t, P]),
    "d2mi_stem_pool": (c_int, [P, P, c_int, c_int, c_int, c_int, P, P]),
    "d2mi_stem_conv": (c_int, [P, P, c_int, c_int, c_int, P, P]),
    "d2mi_preprocess_images": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    "d2mi_roi_gt_classes": (c_int, [P, P, P, c_int, P, c_int, c_int, c_int, c_int, P, P]),
    "d2mi_roi_sample_take": (c_int, [P, P, P, P, P, P] + [c_int] * 6 + [P] * 13),
    "d2mi_rpn_loss_blocks": (c_int, []),
    "d2mi_rpn_loss_fwd": (c_int, [P, P, P, P, P, P, P, c_int, c_int, c_int, P, c_float, P, P]),
    "d2mi_rpn_loss_bwd": (c_int, [P, P, P, P, P, P, P, c_int, c_int, c_int, P, c_float, P, P, P,
                                  P]),
    "d2mi_rpn_loss_bwd_ex": (c_int, [P, P, P, P, P, P, P, c_int, c_int, c_int, P, c_float, P, P,
                                     c_float, P, P, P]),
    "d2mi_fast_rcnn_loss_workspace_size": (c_size_t, [c_int]),
    "d2mi_fast_rcnn_loss_fwd": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, P, c_float, P, P,
                                        c_size_t, P]),
    "d2mi_fast_rcnn_loss_bwd": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, P, c_float, P, P,
                                        P, P, P]),
    "d2mi_mask_loss_workspace_size": (c_size_t, [c_int]),
    "d2mi_mask_loss_fwd": (c_int, [P, P, P, P, c_int, c_int, c_int, P, P, c_size_t, P]),
    "d2mi_mask_loss_bwd": (c_int, [P, P, P, P, c_int, c_int, c_int, P, P, P, P]),
    "d2mi_sgd_table_sizes": (c_int, [P, P, P]),
    "d2mi_momentum_sgd": (c_int, [P, P, c_int, P, c_float, c_float, c_float, P]),
    "d2mi_momentum_sgd_ex": (c_int, [P, P, c_int, P, c_float, c_float, c_float, P, P]),
    "d2mi_retina_loss_blocks": (c_int, []),
    "d2mi_retina_loss_fwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, P, P, c_int, P, P,
                                     c_float, c_float, c_float, P, P, P]),
    "d2mi_retina_loss_bwd": (c_int, [P, P, P, P, P, c_int, c_int, c_int, c_int, P, P, P, c_int, P,
                                     P, c_float, c_float, c_float, P, P, P, P]),
    "d2mi_fold_many_sizes": (c_int, [P, P]),
    "d2mi_fold_frozen_bn_many": (c_int, [P, c_int, c_int, P]),
    "d2mi_fold_frozen_bn_bwd_many": (c_int, [P, c_int, c_int, c_int, P, P]),
}

EXPORTED = tuple(_SIGS)


class D2MIError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load the library (idempotent).  Raises if it is missing or incomplete."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        _load_error = f"{path} not found; run detectron2_tensorflow_amd._build.build()"
        raise D2MIError(_load_error)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)  # AttributeError if the export is missing
        fn.restype = res
        fn.argtypes = args
    # the library must be built from the sources next to it (a stale prebuilt
    # .so would silently run other kernels than the tree's)
    from . import _build
    if os.path.isdir(_build.CSRC) and os.environ.get("D2MI_LIB") is None:
        want, got = _build.source_hash(), lib.d2mi_source_hash().decode()
        if got != want:
            _load_error = (f"{path} was built from other sources (hash {got}, tree {want}); "
                           "rebuild with detectron2_tensorflow_amd._build.build()")
            raise D2MIError(_load_error)
    _lib = lib
    return lib


def lib():
    return _lib if _lib is not None else load()


def last_error():
    msg = lib().d2mi_last_error()
    return msg.decode() if msg else ""


def check(rc, what):
    if rc != 0:
        raise D2MIError(f"{what} failed (rc={rc}): {last_error()}")


def ptr(t):
    """Device pointer of a tensor as a plain int (None -> NULL); ctypes
    converts it for the c_void_p argument without a wrapper object."""
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(device=None):
    """hipStream_t (as an int) of the current torch stream on ``device``."""
    if _raw_stream is not None:
        idx = device.index if isinstance(device, torch.device) else device
        if idx is None:
            idx = torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream


def require_device(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise ValueError(
                "detectron2_tensorflow_amd hot-path ops run on the MI355X only: "
                f"got a tensor on {t.device}")


def host_array(ctype, values):
    arr = (ctype * len(values))(*values)
    return arr


def workspace(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


_scratch = {}
# every scratch buffer ever handed out stays allocated: a launch captured into
# a hipGraph keeps its buffer's address, so a buffer outgrown later (a larger
# request, e.g. a graph of a larger mask-branch row count) must not be freed
# -- torch.cuda.graph's empty_cache() would return it to the driver and the
# earlier graphs' replays would fault on it
_scratch_outgrown = []


def scratch(nbytes, device):
    """A grow-only per-(device, stream) scratch buffer for workspaces that live
    only inside one C call (split-K partials, reductions): every use is
    ordered on that stream, so consecutive calls can share it without an
    allocation each.  Never hand it to anything that outlives the call."""
    idx = device.index if isinstance(device, torch.device) else device
    if idx is None:
        idx = torch.cuda.current_device()
    key = (idx, stream_of(idx))
    buf = _scratch.get(key)
    n = max(int(nbytes), 1)
    if buf is None or buf.numel() < n:
        if buf is not None:
            _scratch_outgrown.append(buf)
        # (grown geometrically: few outgrown buffers)
        size = max(n, 1 << 20, 2 * buf.numel() if buf is not None else 0)
        buf = torch.empty(size, dtype=torch.uint8, device=torch.device("cuda", idx))
        _scratch[key] = buf
    return buf


_ERR_BITS = {1: "box index out of range", 2: "NMS candidate capacity exceeded",
             4: "top-k candidate capacity exceeded"}


def error_word(device=None):
    """Read (synchronising) and decode the device error word."""
    addr = lib().d2mi_error_word_dev()
    if not addr:
        raise D2MIError("cannot resolve the device error word")
    host = ctypes.c_int32(0)
    torch.cuda.synchronize(device)
    # hipMemcpy through torch: wrap the raw device int in a 1-element tensor view
    buf = torch.empty(1, dtype=torch.int32, device=device or "cuda")
    _copy_word(addr, buf)
    v = int(buf.item())
    return v, [m for b, m in _ERR_BITS.items() if v & b]


def _copy_word(addr, dst):
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.restype = ctypes.c_int
    hip.hipMemcpy.argtypes = [c_void_p, c_void_p, c_size_t, c_int]
    rc = hip.hipMemcpy(c_void_p(dst.data_ptr()), c_void_p(addr), 4, 3)  # DeviceToDevice
    if rc != 0:
        raise D2MIError(f"hipMemcpy of the error word failed ({rc})")


def clear_errors(device=None):
    check(lib().d2mi_clear_errors(stream_of(device)), "d2mi_clear_errors")


def raise_on_errors(device=None):
    v, msgs = error_word(device)
    if v:
        clear_errors(device)
        raise D2MIError("device-side error(s): " + ", ".join(msgs))
