"""torch-facing wrappers of the libd2mi_hip.so hot-path kernels.

Every function here launches hand-written HIP on torch's current stream and
raises if the library is missing or a tensor is not on the GPU: there is no
CPU/eager fallback for the hot path.  Shapes and argument meaning follow the
reference op they replace (cited per function).
"""
import math
import os

import numpy as np
import torch

from .. import _C
from ..utils import capture, host_sync
from . import handoff

_DEFAULT_SCALE_CLAMP = math.log(1000.0 / 16)  # lib/modeling/box_regression.py:10

BOX_MODE_RAW, BOX_MODE_ALIGNED, BOX_MODE_UNALIGNED = 0, 1, 2


class KernelTimer:
    """Opt-in per-launch HIP-event timing of the hot kernels (bench.py's live
    roofline).  Events are recorded on the launching stream around each call;
    ``work`` is the op's ALGORITHMIC flops (conv) or bytes (ROIAlign)."""

    enabled = False
    detail = False   # also key records by shape (tools/conv_shapes.py)
    records = []

    @classmethod
    def reset(cls, enabled=True, detail=False):
        cls.enabled = enabled
        cls.detail = detail
        cls.records = []

    @classmethod
    def start(cls):
        if not cls.enabled:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream())
        return ev

    @classmethod
    def stop(cls, ev0, name, work, extra=None):
        """extra: None or a zero-argument callable returning {key: amount} of
        further work models for this launch (evaluated after the timed region,
        by extras())."""
        if ev0 is None:
            return
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record(torch.cuda.current_stream())
        cls.records.append((name, ev0, ev1, float(work), extra))

    @classmethod
    def summary(cls):
        """{name: (launches, total_ms, total_work)} (synchronises)."""
        torch.cuda.synchronize()
        out = {}
        for name, e0, e1, w, _ in cls.records:
            n, t, tw = out.get(name, (0, 0.0, 0.0))
            out[name] = (n + 1, t + e0.elapsed_time(e1), tw + w)
        return out

    @classmethod
    def extras(cls):
        """{name: {key: total}} of the launches' extra work models."""
        out = {}
        for name, _, _, _, ex in cls.records:
            if ex is None:
                continue
            d = out.setdefault(name, {})
            for k, v in ex().items():
                d[k] = d.get(k, 0.0) + float(v)
        return out


def roi_touched_rows(boxes, box_ind, params, shapes, return_ids=False):
    """Distinct feature rows (level, image, y, x) that one ROIAlign forward
    reads (the 4 bilinear corners of every in-range sample): the unique-bytes
    model of bench.py's roofline (rows x C x 4 bytes is the least HBM
    traffic that can deliver the launch's inputs, however many samples share
    a row).  A float32 torch restatement of roi_geom / make_tap in
    csrc/roi_align.hip, for the byte count only (a log-boundary box may land
    on the other level here: immaterial for a traffic model)."""
    (oh, ow, scales, sr, mode, pad, assign, min_l, max_l, canon_s, canon_l, _) = params
    dev = boxes.device
    b = boxes.detach().float().reshape(-1, 4)
    R = b.shape[0]
    if R == 0:
        return torch.zeros(0, dtype=torch.long, device=dev) if return_ids else 0
    if assign and len(shapes) > 1:
        area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
        v = canon_l + torch.log(torch.sqrt(area) / canon_s + 2.220446049250313e-16) / math.log(2)
        lv = torch.nan_to_num(torch.floor(v), nan=min_l).clamp(min_l, max_l).long() - min_l
    else:
        lv = torch.zeros(R, dtype=torch.long, device=dev)
    Hs = torch.tensor([s[1] for s in shapes], device=dev)[lv]
    Ws = torch.tensor([s[2] for s in shapes], device=dev)[lv]
    sc = torch.tensor(list(scales), dtype=torch.float32, device=dev)[lv]
    S = max(sr, 1)
    ch, cw = oh * S, ow * S
    y1, x1, y2, x2 = b.unbind(1)
    if mode != BOX_MODE_RAW:
        y1, x1, y2, x2 = y1 * sc, x1 * sc, y2 * sc, x2 * sc
    Hp, Wp = (Hs + 2, Ws + 2) if pad else (Hs, Ws)
    if pad:
        y1, x1, y2, x2 = y1 + 1, x1 + 1, y2 + 1, x2 + 1
    i0, i1 = (Hp - 1).float(), (Wp - 1).float()
    if mode == BOX_MODE_ALIGNED:
        sh, sw = (y2 - y1) / ch, (x2 - x1) / cw
        ny, nx = (y1 + sh / 2 - 0.5) / i0, (x1 + sw / 2 - 0.5) / i1
        y1, x1, y2, x2 = ny, nx, ny + sh * (ch - 1) / i0, nx + sw * (cw - 1) / i1
    elif mode == BOX_MODE_UNALIGNED:
        y1, y2, x1, x2 = y1 / Hp.float(), y2 / Hp.float(), x1 / Wp.float(), x2 / Wp.float()

    def taps(c1, c2, img_p, img, crop):
        i = torch.arange(crop, device=dev, dtype=torch.float32)
        if crop > 1:
            pos = c1[:, None] * (img_p - 1).float()[:, None] + i * (
                (c2 - c1) * (img_p - 1).float() / (crop - 1))[:, None]
        else:
            pos = (0.5 * (c1 + c2) * (img_p - 1).float())[:, None]
        ok = (pos >= 0) & (pos <= (img_p - 1).float()[:, None])
        lo, hi = torch.floor(pos).long(), torch.ceil(pos).long()
        d = 1 if pad else 0
        top = img[:, None] - 1
        return ok, (lo - d).clamp(min=0).minimum(top), (hi - d).clamp(min=0).minimum(top)

    oky, ylo, yhi = taps(y1, y2, Hp, Hs, ch)
    okx, xlo, xhi = taps(x1, x2, Wp, Ws, cw)
    n = box_ind.detach().long().reshape(-1)
    base = torch.tensor([0] + [s[0] * s[1] * s[2] for s in shapes], device=dev).cumsum(0)
    img0 = (base[lv] + n * Hs * Ws)[:, None, None]
    ok = (oky[:, :, None] & okx[:, None, :]).reshape(-1)
    ids = []
    for yy in (ylo, yhi):
        for xx in (xlo, xhi):
            ids.append((img0 + yy[:, :, None] * Ws[:, None, None] + xx[:, None, :]).reshape(-1)[ok])
    u = torch.unique(torch.cat(ids))
    return u if return_ids else int(u.numel())


def get_tuning(key):
    """d2mi_get_tuning: the knob's current value."""
    v = _C.lib().d2mi_get_tuning(key.encode())
    if v == -2 ** 31:
        raise KeyError(f"unknown tuning key {key!r}")
    return v


def set_tuning(key, value):
    """d2mi_set_tuning (in-process A/B of kernel variants, tools/); clears the
    conv workspace-size cache, whose plans may depend on the knob."""
    _C.check(_C.lib().d2mi_set_tuning(key.encode(), int(value)), "d2mi_set_tuning")
    _CONV_WS.clear()
    _WGRAD_WS.clear()


def _f32c(t):
    if t.dtype is torch.float32 and t.is_contiguous():
        return t
    return t.to(torch.float32).contiguous()


def _i32c(t):
    if t.dtype is torch.int32 and t.is_contiguous():
        return t
    return t.to(torch.int32).contiguous()


# ------------------------------------------------------------------ ROIAlign
class _RoIAlignFn(torch.autograd.Function):
    """ROIAlign forward/backward over 1..8 feature levels.  Boxes carry no
    gradient (crop_and_resize stop_gradient, lib/layers/functional.py:120).

    grad_share (a dict shared by two poolings of the SAME feature maps, the
    box and mask poolers of a training step, both of whose backwards always
    run): the first backward writes the full maps and leaves them in the
    dict, returning no gradient for the features; the second adds its
    contributions into them (d2mi_roi_align_bwd_ex accumulate: no second
    183 MB clear at 1333x800, no autograd add of two maps) and returns the
    sum — bit-identical to autograd's add of the two maps."""

    @staticmethod
    def forward(ctx, boxes, box_ind, params, grad_share, *feats):
        feats = [_f32c(f) for f in feats]
        boxes = _f32c(boxes)
        box_ind = _i32c(box_ind)
        _C.require_device(boxes, box_ind, *feats)
        (out_h, out_w, scales, sr, mode, pad, assign, min_l, max_l, canon_s, canon_l,
         want_level) = params
        L = len(feats)
        C = feats[0].shape[-1]
        R = boxes.shape[0]
        out = torch.empty((R, out_h, out_w, C), dtype=torch.float32, device=boxes.device)
        level = torch.empty((R,), dtype=torch.int32, device=boxes.device) if want_level else None
        fp = _C.host_array(_C.c_void_p, [f.data_ptr() for f in feats])
        dims = _C.host_array(_C.ctypes.c_int32,
                             [v for f in feats for v in (f.shape[0], f.shape[1], f.shape[2])])
        sc = _C.host_array(_C.c_float, list(scales))
        ev = KernelTimer.start()
        rc = _C.lib().d2mi_roi_align_fwd(fp, dims, sc, L, C, _C.ptr(boxes), _C.ptr(box_ind), R,
                                         out_h, out_w, sr, mode, pad, assign, min_l, max_l,
                                         canon_s, canon_l, _C.ptr(level), _C.ptr(out),
                                         _C.stream_of(boxes.device))
        S = max(sr, 1) ** 2
        # algorithmic bytes: 4 f32 corner reads per sample + 1 f32
        # write per output.  Feature-pyramid pooling (C >= 64, the hot path) and
        # narrow crops (the C = 1 mask-target crop_and_resize) are timed apart,
        # and the box pooler (7x7) apart from the mask pooler (14x14, a few
        # dozen ROIs per step: latency-bound)
        name = ("crop_and_resize_fwd_narrow" if C < 64 else
                "roi_align_fwd" if out_h * out_w <= 49 else "roi_align_fwd_mask")
        shapes = [tuple(f.shape) for f in feats]
        KernelTimer.stop(ev, name, R * out_h * out_w * C * (16 * S + 4),
                         extra=lambda: {"unique_bytes": C * 4 * (
                             roi_touched_rows(boxes, box_ind, params, shapes) + R * out_h * out_w)})
        _C.check(rc, "d2mi_roi_align_fwd")
        ctx.params = params
        ctx.share = grad_share
        ctx.shapes = [f.shape for f in feats]
        # per-level input-gradient hand-off with another consumer of the same
        # maps (the RPN head conv: ops / convolutional pair_grad protocol)
        ctx.pairs = [getattr(f, "_d2mi_grad_pair", None) for f in feats]
        ctx.save_for_backward(boxes, box_ind)
        ctx.set_materialize_grads(False)  # level (non-differentiable): no zero grad
        if level is not None:
            ctx.mark_non_differentiable(level)
        return out, level

    @staticmethod
    def backward(ctx, grad_out, _grad_level):
        if grad_out is None:
            return (None,) * (4 + len(ctx.shapes))
        boxes, box_ind = ctx.saved_tensors
        (out_h, out_w, scales, sr, mode, pad, assign, min_l, max_l, canon_s, canon_l,
         _) = ctx.params
        share = ctx.share
        if share is not None and MERGED_BWD and grad_out.shape[-1] >= 64:
            # a pair of poolings of the same maps: the first backward only
            # leaves its grad_out; the second runs ONE backward over both ROI
            # sets (one emit per set, one sort, one gather pass summing each
            # set's run apart, set 0 + set 1)
            first = share.pop("set0", None)
            g = _f32c(grad_out)
            if first is None:
                handoff.deposit(share, "set0", (boxes, box_ind, g, ctx.params), "box/mask poolers")
                return (None,) * (4 + len(ctx.shapes))
            # levels whose other consumer already left its input gradient:
            # accumulate into it; the others: their pixel pass is deferred
            # into that consumer's backward, which writes the level's full
            # map (DEFER_PIXELS), or the map is written here and left for it
            given = [pr.pop("g", None) if pr is not None else None for pr in ctx.pairs]
            defer = [DEFER_PIXELS and pr is not None and gv is None
                     for pr, gv in zip(ctx.pairs, given)]
            grads = _roi_align_bwd2(first, (boxes, box_ind, g, ctx.params), ctx.shapes, given,
                                    defer)
            out = []
            for pr, gv, gr in zip(ctx.pairs, given, grads):
                if pr is not None and gv is None:
                    # the other consumer adds it: a deferred pixel pass into its
                    # dgrad, or the map in its dgrad epilogue
                    handoff.deposit(pr, "g", gr, "RPN head / ROI pooler level")
                    out.append(None)
                else:
                    out.append(gr)
            return (None, None, None, None, *out)
        prior = share.pop("maps", None) if share is not None else None
        if prior is not None:  # second of a pair: add into the first's maps
            grads = prior
        else:
            # every element is written by d2mi_roi_align_bwd (zero-fill + touched pixels)
            grads = [torch.empty(s, dtype=torch.float32, device=boxes.device) for s in ctx.shapes]
        g = _f32c(grad_out)
        gp = _C.host_array(_C.c_void_p, [x.data_ptr() for x in grads])
        dims = _C.host_array(_C.ctypes.c_int32, [v for s in ctx.shapes for v in (s[0], s[1], s[2])])
        sc = _C.host_array(_C.c_float, list(scales))
        R, C = boxes.shape[0], ctx.shapes[0][-1]
        wsb = _C.lib().d2mi_roi_align_bwd_workspace_size(dims, len(grads), C, R, out_h, out_w, sr)
        ws = _C.workspace(wsb, boxes.device)
        ev = KernelTimer.start()
        rc = _C.lib().d2mi_roi_align_bwd_ex(gp, dims, sc, len(grads), C, _C.ptr(boxes),
                                            _C.ptr(box_ind), R, out_h, out_w, sr, mode, pad,
                                            assign, min_l, max_l, canon_s, canon_l, _C.ptr(g),
                                            int(prior is not None), _C.ptr(ws), wsb,
                                            _C.stream_of(boxes.device))
        # algorithmic bytes: R*oh*ow*C*(4 + 32*S) = the grad_out read
        # + 4 corner read-modify-writes per sample of the reference's scatter
        S = max(sr, 1) ** 2
        maps = sum(int(np.prod(s)) for s in ctx.shapes) * 4
        KernelTimer.stop(ev, "roi_align_bwd" if C >= 64 else "crop_and_resize_bwd_narrow",
                         R * out_h * out_w * C * (4 + 32 * S),
                         extra=lambda: {"unique_bytes": R * out_h * out_w * C * 4 + maps})
        _C.check(rc, "d2mi_roi_align_bwd")
        if share is not None and prior is None:  # first of a pair: hand the maps over
            handoff.deposit(share, "maps", grads, "box/mask poolers")
            return (None,) * (4 + len(grads))
        return (None, None, None, None, *grads)


# The box and mask poolers' backwards as one merged backward (False: two
# backwards, the second accumulating into the first's maps; tests compare).
MERGED_BWD = True
# r4: a merged backward whose level is also read by another consumer that has
# not run its backward yet (the RPN head conv) prepares the contributions
# once (d2mi_roi_align_bwd2_ex phase 1) and leaves each such level's pixel
# pass (phase 2) to that consumer, which runs it into its own full dgrad map
# (DeferredPixels.add_into): the level's map is neither cleared here nor
# written twice nor read again by the consumer's epilogue.  False: the full
# maps are written here and added in the consumer's dgrad epilogue (A/B).
DEFER_PIXELS = True


class DeferredPixels:
    """The pixel pass of ONE level of a merged ROIAlign backward
    (d2mi_roi_align_bwd2_ex phase 2), deposited for the backward that writes
    that level's full gradient map.  add_into(gx) adds the pooled
    contributions into gx in place (old + new at each touched pixel: the
    rounding of autograd's sum of the two maps); materialize() returns the
    pooled map alone (a fresh zeroed map + the pass), for a consumer that
    cannot take it afterwards."""

    def __init__(self, run, level, shape, device):
        self._run, self.level, self.shape, self.device = run, level, tuple(shape), device

    def add_into(self, gx):
        if (tuple(gx.shape) != self.shape or gx.dtype != torch.float32 or not gx.is_contiguous()
                or gx.device != self.device):
            raise ValueError(f"deferred ROIAlign pixels: need a contiguous f32 {self.shape} map")
        self._run(self.level, gx, True)
        return gx

    def materialize(self):
        m = torch.empty(self.shape, dtype=torch.float32, device=self.device)
        self._run(self.level, m, False)
        return m


def _roi_align_bwd2(set0, set1, shapes, given=None, defer=None):
    """d2mi_roi_align_bwd2 over two (boxes, box_ind, grad_out, params) sets
    of the same feature maps (equal level / box-mode parameters).  given[l]:
    a gradient map of level l to accumulate into (returned), or None.
    defer[l]: level l's pixel pass is left to a DeferredPixels (returned in
    its place; d2mi_roi_align_bwd2_ex phase 1 now, phase 2 later)."""
    b0, i0, g0, p0 = set0
    b1, i1, g1, p1 = set1
    if p0[2] != p1[2] or p0[4:11] != p1[4:11]:  # scales, box mode .. canonical level
        raise ValueError("merged ROIAlign backward: the two poolings differ beyond their crops")
    (oh0, ow0, scales, sr0, mode, pad, assign, min_l, max_l, canon_s, canon_l, _) = p0
    oh1, ow1, sr1 = p1[0], p1[1], p1[3]
    dev = b0.device
    L = len(shapes)
    given = given or [None] * L
    defer = defer or [False] * L
    grads, acc_mask = [], 0
    for l, (s, gv) in enumerate(zip(shapes, given)):
        if defer[l]:
            grads.append(None)
            acc_mask |= 1 << l  # (phase 1 leaves the deferred maps alone)
        elif gv is not None and tuple(gv.shape) == tuple(s) and gv.dtype == torch.float32 \
                and gv.is_contiguous():
            grads.append(gv)
            acc_mask |= 1 << l
        elif gv is not None:
            grads.append(_f32c(gv).clone())
            acc_mask |= 1 << l
        else:
            grads.append(torch.empty(s, dtype=torch.float32, device=dev))
    dims = _C.host_array(_C.ctypes.c_int32, [v for s in shapes for v in (s[0], s[1], s[2])])
    sc = _C.host_array(_C.c_float, list(scales))
    C = shapes[0][-1]
    R0, R1 = b0.shape[0], b1.shape[0]
    lib = _C.lib()
    wsb = lib.d2mi_roi_align_bwd2_workspace_size(dims, L, C, R0, oh0, ow0, sr0, R1, oh1, ow1, sr1)
    ws = _C.workspace(wsb, dev)
    st = _C.stream_of(dev)
    S0, S1 = max(sr0, 1) ** 2, max(sr1, 1) ** 2
    d4 = R0 * oh0 * ow0 * C * (4 + 32 * S0) + R1 * oh1 * ow1 * C * (4 + 32 * S1)
    gout_bytes = (R0 * oh0 * ow0 + R1 * oh1 * ow1) * C * 4

    def touched_bytes(levels):
        """unique bytes of a pixel pass: 2 x C x 4 per touched pixel of these
        levels (read + write of an accumulated map) -- the union of the pixels
        the two sets' sample corners touch (roi_touched_rows)."""
        base = np.cumsum([0] + [int(s[0] * s[1] * s[2]) for s in shapes])
        ids = torch.cat([roi_touched_rows(b, i, p, shapes, return_ids=True)
                         for b, i, _, p in (set0, set1)]).unique()
        lo, hi = int(base[min(levels)]), int(base[max(levels) + 1])
        return 2 * C * 4 * int(((ids >= lo) & (ids < hi)).sum())

    def call(maps, acc, phase, lo, hi):
        gp = _C.host_array(_C.c_void_p, [m.data_ptr() if m is not None else None for m in maps])
        return lib.d2mi_roi_align_bwd2_ex(gp, dims, sc, L, C, mode, pad, assign, min_l, max_l,
                                          canon_s, canon_l, _C.ptr(b0), _C.ptr(i0), R0, oh0, ow0,
                                          sr0, _C.ptr(g0), _C.ptr(b1), _C.ptr(i1), R1, oh1, ow1,
                                          sr1, _C.ptr(g1), acc, phase, lo, hi, _C.ptr(ws), wsb, st)

    ev = KernelTimer.start()
    if not any(defer):
        rc = call(grads, acc_mask, 3, 0, L - 1)
        maps = sum(int(np.prod(s)) for s in shapes) * 4
        # unique-bytes model: both grad_out sets read once + every element of
        # the dense gradient maps written once
        KernelTimer.stop(ev, "roi_align_bwd", d4,
                         extra=lambda: {"unique_bytes": gout_bytes + maps})
        _C.check(rc, "d2mi_roi_align_bwd2")
        return grads
    rc = call(grads, acc_mask, 1, 0, L - 1)
    fresh = [l for l in range(L) if not defer[l]]
    # the prepare launches: the grad_out reads (the contributions' records)
    KernelTimer.stop(ev, "roi_align_bwd", d4, extra=lambda: {"unique_bytes": gout_bytes})
    _C.check(rc, "d2mi_roi_align_bwd2_ex (prepare)")

    def run(level, m, accumulate):
        maps = [None] * L
        maps[level] = m
        ev = KernelTimer.start()
        rc = call(maps, (1 << level) if accumulate else 0, 2, level, level)
        KernelTimer.stop(ev, "roi_align_bwd", 0.0,
                         extra=lambda: {"unique_bytes": touched_bytes([level])})
        _C.check(rc, "d2mi_roi_align_bwd2_ex (pixels)")

    for l in fresh:  # levels without a deferral: their passes now (maps zeroed or given)
        run(l, grads[l], True)
    for l in range(L):
        if defer[l]:
            grads[l] = DeferredPixels(run, l, shapes[l], dev)
    return grads


def roi_align(features, boxes, box_ind, output_size, scales, sampling_ratio=0, aligned=True,
              pad_border=True, assign_levels=True, min_level=None, max_level=None,
              canonical_box_size=224, canonical_level=4, return_levels=False,
              box_mode=None, grad_share=None):
    """Multi-level ROIAlign (poolers.py:134-180 + roi_align.py:45-66 +
    functional.py:100-166) in one launch; output rows in input order.
    grad_share: see _RoIAlignFn (two poolings of one set of maps)."""
    if not isinstance(features, (list, tuple)):
        features = [features]
    L = len(features)
    if min_level is None:
        min_level = int(round(-math.log2(scales[0]))) if L > 1 else 0
        max_level = int(round(-math.log2(scales[-1]))) if L > 1 else 0
    if box_mode is None:
        box_mode = BOX_MODE_ALIGNED if aligned else BOX_MODE_UNALIGNED
    oh, ow = (output_size, output_size) if isinstance(output_size, int) else output_size
    params = (int(oh), int(ow), tuple(float(s) for s in scales), int(sampling_ratio),
              int(box_mode), int(bool(pad_border)), int(bool(assign_levels and L > 1)),
              int(min_level), int(max_level), int(canonical_box_size), int(canonical_level),
              bool(return_levels))
    out, level = _RoIAlignFn.apply(boxes, box_ind, params, grad_share, *features)
    return (out, level) if return_levels else out


# ----------------------------------------------------------------------- NMS
def nms_segments(boxes, scores, seg_offsets, max_output_size, iou_threshold, seg_capacity=None):
    """Segmented TF NonMaxSuppressionV3.  boxes [T,4], scores [T], seg_offsets
    int [S+1] (device).  Returns keep [S, max_out] int32 (segment-relative,
    -1 padded) and num_keep [S] int32."""
    if not 0.0 <= float(iou_threshold) <= 1.0:
        raise ValueError("iou_threshold must be in [0, 1], got %r" % (iou_threshold,))
    if max_output_size < 0:
        raise ValueError("max_output_size must be non-negative, got %r" % (max_output_size,))
    boxes, scores, seg_offsets = _f32c(boxes), _f32c(scores), _i32c(seg_offsets)
    _C.require_device(boxes, scores, seg_offsets)
    S = seg_offsets.shape[0] - 1
    if seg_capacity is None:
        seg_capacity = int(boxes.shape[0])
    dev = boxes.device
    keep = torch.empty((S, max(int(max_output_size), 1)), dtype=torch.int32, device=dev)
    num = torch.empty((S,), dtype=torch.int32, device=dev)
    wsb = _C.lib().d2mi_nms_workspace_size(S, int(seg_capacity))
    ws = _C.workspace(wsb, dev)
    rc = _C.lib().d2mi_nms(_C.ptr(boxes), _C.ptr(scores), _C.ptr(seg_offsets), S,
                           int(seg_capacity), int(max_output_size), float(iou_threshold),
                           _C.ptr(keep), _C.ptr(num), _C.ptr(ws), wsb, _C.stream_of(dev))
    _C.check(rc, "d2mi_nms")
    return keep[:, :max_output_size], num


def non_max_suppression(boxes, scores, max_output_size, iou_threshold=0.5):
    """tf.image.non_max_suppression: selected indices (int32, selection order)."""
    n = boxes.shape[0]
    off = torch.tensor([0, n], dtype=torch.int32, device=boxes.device)
    keep, num = nms_segments(boxes, scores, off, max_output_size, iou_threshold, seg_capacity=n)
    return keep[0, : int(num[0].item())]


# --------------------------------------------------------------------- top-k
TOPK_MAX_K = 8192  # d2mi_topk's largest k (kCap in csrc/topk.hip)


def topk_segments(values, seg_start, seg_len, k, max_seg_len, sigmoid=False):
    """Exact segmented top-k (tf.nn.top_k sorted=True order)."""
    values = _f32c(values)
    seg_start = seg_start.to(torch.int64).contiguous()
    seg_len = _i32c(seg_len)
    _C.require_device(values, seg_start, seg_len)
    S = seg_len.shape[0]
    dev = values.device
    vals = torch.empty((S, max(k, 1)), dtype=torch.float32, device=dev)
    idx = torch.empty((S, max(k, 1)), dtype=torch.int32, device=dev)
    cnt = torch.empty((S,), dtype=torch.int32, device=dev)
    wsb = _C.lib().d2mi_topk_workspace_size(S, k)
    ws = _C.workspace(wsb, dev)
    rc = _C.lib().d2mi_topk(_C.ptr(values), _C.ptr(seg_start), _C.ptr(seg_len), S,
                            int(max_seg_len), int(k), int(bool(sigmoid)), _C.ptr(vals),
                            _C.ptr(idx), _C.ptr(cnt), _C.ptr(ws), wsb, _C.stream_of(dev))
    _C.check(rc, "d2mi_topk")
    return vals[:, :k], idx[:, :k], cnt


def subsample(labels, num_samples, num_pos, bg_label, seed, order_slots=0):
    """d2mi_subsample: (pos, neg) [N, P] bool -- a uniformly random
    min(num_pos, #pos) positives and min(num_samples - that, #neg) negatives
    per row (labels int64: -1 ignore, bg_label negative, else positive);
    with order_slots = S also (order [N, S] int64, valid [N, S] bool): the
    selected indices positives first, each kind in index order.  seed: a
    device int64 tensor [1]."""
    if labels.dtype is not torch.int64 or not labels.is_contiguous():
        labels = labels.to(torch.int64).contiguous()
    _C.require_device(labels, seed)
    N, P = labels.shape
    dev = labels.device
    # bool outputs written directly (one byte, 0 / 1: the kernel's uint8)
    pos = torch.empty((N, P), dtype=torch.bool, device=dev)
    neg = torch.empty((N, P), dtype=torch.bool, device=dev)
    S = int(order_slots)
    order = torch.empty((N, S), dtype=torch.int64, device=dev) if S else None
    valid = torch.empty((N, S), dtype=torch.bool, device=dev) if S else None
    wsb = _C.lib().d2mi_subsample_workspace_size(N, P)
    ws = _C.workspace(wsb, dev)
    rc = _C.lib().d2mi_subsample(_C.ptr(labels), N, P, int(bg_label), int(num_samples),
                                 int(num_pos), _C.ptr(seed), _C.ptr(pos), _C.ptr(neg),
                                 _C.ptr(order), _C.ptr(valid), S, _C.ptr(ws), wsb,
                                 _C.stream_of(dev))
    _C.check(rc, "d2mi_subsample")
    if S:
        return pos, neg, order, valid
    return pos, neg


# The ROI heads' label / take / mask-prep glue on d2mi_roi_gt_classes and
# d2mi_roi_sample_take (False: torch's gathers, selects, argsort; tests compare;
# D2MI_FUSED_SAMPLE_TAKE=0 for a bench A/B).
FUSED_SAMPLE_TAKE = os.environ.get("D2MI_FUSED_SAMPLE_TAKE", "1") != "0"


def roi_gt_classes(labels, matches, gt_classes, pvalid, num_classes):
    """d2mi_roi_gt_classes: the training class of every proposal, [N, M] int64
    (roi_heads.py:160-216): the matched GT class for label 1, num_classes
    (background) for 0, -1 for ignored rows and invalid proposal slots."""
    _C.require_device(labels, matches, gt_classes, pvalid)
    if labels.dtype is not torch.int64 or matches.dtype is not torch.int64:
        raise ValueError("roi_gt_classes: labels / matches must be int64")
    labels, matches = labels.contiguous(), matches.contiguous()
    if gt_classes.dtype not in (torch.int32, torch.int64):
        gt_classes = gt_classes.to(torch.int64)
    gt_classes = gt_classes.contiguous()
    pv = pvalid.to(torch.bool).contiguous()
    N, M = labels.shape
    G = gt_classes.shape[1]
    out = torch.empty((N, M), dtype=torch.int64, device=labels.device)
    rc = _C.lib().d2mi_roi_gt_classes(_C.ptr(labels), _C.ptr(matches), _C.ptr(gt_classes),
                                      int(gt_classes.dtype is torch.int64), _C.ptr(pv), N, M, G,
                                      int(num_classes), _C.ptr(out), _C.stream_of(labels.device))
    _C.check(rc, "d2mi_roi_gt_classes")
    return out


def roi_sample_take(order, valid, boxes, gt_classes, matches, gt_boxes, num_classes, mask_slots):
    """d2mi_roi_sample_take: the sampled dict of label_and_sample_proposals
    (boxes, gt_classes, gt_index, gt_boxes [N, S(, 4)]) and, mask_slots = F >
    0, the mask branch's inputs over the first F slots per image in stable
    foreground-first order: ((boxes, classes, fg, image, mask index, gt boxes),
    fg [N*F] in slot order, count [1] int64)."""
    _C.require_device(order, valid, boxes, gt_classes, matches, gt_boxes)
    order, valid = order.contiguous(), valid.to(torch.bool).contiguous()
    boxes, gt_boxes = _f32c(boxes), _f32c(gt_boxes)
    gt_classes, matches = gt_classes.contiguous(), matches.contiguous()
    N, S = order.shape
    M, G, F = boxes.shape[1], gt_boxes.shape[1], int(mask_slots)
    dev = order.device
    s_boxes = torch.empty((N, S, 4), dtype=torch.float32, device=dev)
    s_cls = torch.empty((N, S), dtype=torch.int64, device=dev)
    s_gidx = torch.empty((N, S), dtype=torch.int64, device=dev)
    s_gtb = torch.empty((N, S, 4), dtype=torch.float32, device=dev)
    R = N * F
    m = None
    if F:
        m = (torch.empty((R, 4), dtype=torch.float32, device=dev),
             torch.empty((R,), dtype=torch.int64, device=dev),
             torch.empty((R,), dtype=torch.bool, device=dev),
             torch.empty((R,), dtype=torch.int32, device=dev),
             torch.empty((R,), dtype=torch.int64, device=dev),
             torch.empty((R, 4), dtype=torch.float32, device=dev),
             torch.empty((R,), dtype=torch.bool, device=dev),
             torch.empty((1,), dtype=torch.int64, device=dev))
    mp = [_C.ptr(t) for t in m] if m else [None] * 8
    rc = _C.lib().d2mi_roi_sample_take(_C.ptr(order), _C.ptr(valid), _C.ptr(boxes),
                                       _C.ptr(gt_classes), _C.ptr(matches), _C.ptr(gt_boxes), N,
                                       M, S, G, F, int(num_classes), _C.ptr(s_boxes),
                                       _C.ptr(s_cls), _C.ptr(s_gidx), _C.ptr(s_gtb), *mp,
                                       _C.stream_of(dev))
    _C.check(rc, "d2mi_roi_sample_take")
    sampled = {"boxes": s_boxes, "gt_classes": s_cls, "gt_index": s_gidx, "gt_boxes": s_gtb,
               "is_valid": valid}
    return sampled, ((m[:6], m[6], m[7]) if m else None)


# ------------------------------------------------------------ anchors/deltas
def grid_anchors(H, W, stride, cell_anchors, device):
    """DefaultAnchorGenerator.grid_anchors for one level -> [H*W*A, 4]."""
    cell = [float(v) for v in torch.as_tensor(cell_anchors, dtype=torch.float32).reshape(-1)]
    A = len(cell) // 4
    out = torch.empty((H * W * A, 4), dtype=torch.float32, device=device)
    rc = _C.lib().d2mi_grid_anchors(int(H), int(W), float(stride),
                                    _C.host_array(_C.c_float, cell), A, _C.ptr(out),
                                    _C.stream_of(device))
    _C.check(rc, "d2mi_grid_anchors")
    return out


def apply_deltas(deltas, boxes, weights, scale_clamp=_DEFAULT_SCALE_CLAMP):
    """Box2BoxTransform.apply_deltas: deltas [N, K*4], boxes [N, 4]."""
    deltas, boxes = _f32c(deltas), _f32c(boxes)
    _C.require_device(deltas, boxes)
    N = boxes.shape[0]
    K = deltas.shape[1] // 4
    out = torch.empty_like(deltas)
    if N == 0:
        return out
    rc = _C.lib().d2mi_apply_deltas(_C.ptr(deltas), _C.ptr(boxes), N, K,
                                    _C.host_array(_C.c_float, [float(w) for w in weights]),
                                    float(scale_clamp), _C.ptr(out), _C.stream_of(boxes.device))
    _C.check(rc, "d2mi_apply_deltas")
    return out


# -------------------------------------------------------------------- convs
def pack_conv_weights(w_hwio):
    """HWIO -> [KH, KW, Cout, Cin] for d2mi_conv2d_nhwc."""
    w = _f32c(w_hwio)
    _C.require_device(w)
    KH, KW, Cin, Cout = w.shape
    out = torch.empty((KH, KW, Cout, Cin), dtype=torch.float32, device=w.device)
    rc = _C.lib().d2mi_conv_pack_weights(_C.ptr(w), KH, KW, Cin, Cout, _C.ptr(out),
                                         _C.stream_of(w.device))
    _C.check(rc, "d2mi_conv_pack_weights")
    return out


def pack_conv_weights_many(ws):
    """pack_conv_weights of every HWIO tensor in ``ws`` (d2mi_conv_pack_weights_many:
    one launch for all Cin % 64 == 0 tensors); bit-identical copies."""
    ws = [_f32c(w) for w in ws]
    if not ws:
        return []
    _C.require_device(*ws)
    outs = [torch.empty((w.shape[0], w.shape[1], w.shape[3], w.shape[2]), dtype=torch.float32,
                        device=w.device) for w in ws]
    wp = _C.host_array(_C.c_void_p, [w.data_ptr() for w in ws])
    op = _C.host_array(_C.c_void_p, [o.data_ptr() for o in outs])
    dims = _C.host_array(_C.ctypes.c_int32, [int(v) for w in ws for v in w.shape])
    rc = _C.lib().d2mi_conv_pack_weights_many(len(ws), wp, dims, op, _C.stream_of(ws[0].device))
    _C.check(rc, "d2mi_conv_pack_weights_many")
    return outs


# Conv MFMA product form: "f32" = v_mfma_f32_32x32x2_f32 (exact f32 products);
# "split" = the same f32 operands split exactly into three bf16 terms
# (h + m + l == x) and multiplied with six v_mfma_f32_32x32x16_bf16 products
# (f32-class error, see csrc/conv_mfma.hip), split while the kernel stages
# its tiles.  Process-wide default from D2MI_CONV_MATH.
CONV_MATH = os.environ.get("D2MI_CONV_MATH", "split")


def split_bf16x3(x):
    """f32 tensor -> int16 [3, *x.shape]: bf16 bit patterns of the exact split
    x = h + m + l (truncation; csrc/conv_mfma.hip split3)."""
    x = _f32c(x)
    _C.require_device(x)
    if x.numel() % 4:
        raise ValueError("split_bf16x3: numel must be a multiple of 4")
    out = torch.empty((3,) + tuple(x.shape), dtype=torch.int16, device=x.device)
    rc = _C.lib().d2mi_split_bf16x3(_C.ptr(x), x.numel(), _C.ptr(out), _C.stream_of(x.device))
    _C.check(rc, "d2mi_split_bf16x3")
    return out


# workspace sizes per conv / wgrad shape (pure functions of the shape and the
# device's CU count: one ctypes query per distinct shape)
_CONV_WS, _WGRAD_WS = {}, {}


# Narrow-Cout convs (<= 64: the 128x64 / 128x32 tiles) run the split-product
# kernel too (r2 A/B, tools/conv_ab.py: res2 3x3 64->64 125 -> 103 us, 1x1
# 256->64 71 -> 61 us, 512->64 46 -> 34 us vs the native f32 MFMA);
# D2MI_NARROW_SPLIT=0 puts them back on the f32 kernel.
_NARROW_SPLIT = os.environ.get("D2MI_NARROW_SPLIT", "1") != "0"


def conv2d_nhwc(x, w_packed, bias=None, stride=1, pad=(0, 0), relu=False, topdown=None,
                residual=None, relu_after_add=False, math_mode=None, flip_taps=False,
                relu_gate=None, out=None):
    """MFMA implicit-GEMM conv: x [N,H,W,Cin], w_packed [KH,KW,Cout,Cin].
    relu_after_add: relu(conv + bias + residual/topdown) instead of
    relu(conv + bias) + residual/topdown.  math_mode: "f32" | "split" (None:
    CONV_MATH).  flip_taps: use the spatially flipped kernel (w_packed[KH-1-i, KW-1-j]).
    relu_gate: a ReLU output of the result's shape: out = gate > 0 ? conv
    (+ residual) : 0 (a dgrad with its producer's ReLU backward fused, and the
    gradient of the producer's other consumer added first)."""
    math_mode = math_mode or CONV_MATH
    if math_mode not in ("f32", "split"):
        raise ValueError(f"conv math must be 'f32' or 'split', got {math_mode!r}")
    x = _f32c(x)
    _C.require_device(x, w_packed)
    N, H, W, Cin = x.shape
    KH, KW, Cout, Cin2 = w_packed.shape
    if Cin != Cin2:
        raise ValueError(f"conv input has {Cin} channels, weights expect {Cin2}")
    pb, pe = pad
    OH = (H + pb + pe - KH) // stride + 1
    OW = (W + pb + pe - KW) // stride + 1
    if out is not None:
        if (tuple(out.shape) != (N, OH, OW, Cout) or out.dtype != torch.float32
                or not out.is_contiguous() or out.device != x.device):
            raise ValueError(f"out must be a contiguous f32 {(N, OH, OW, Cout)} tensor on {x.device}")
        y = out
    else:
        y = torch.empty((N, OH, OW, Cout), dtype=torch.float32, device=x.device)
    if topdown is not None:
        topdown = _f32c(topdown)
        if topdown.shape != (N, (OH + 1) // 2, (OW + 1) // 2, Cout):
            raise ValueError(f"top-down map {tuple(topdown.shape)} does not upsample to "
                             f"{(N, OH, OW, Cout)}")
    if residual is not None:
        residual = _f32c(residual)
    if relu_gate is not None:
        if topdown is not None or relu:
            raise ValueError("relu_gate excludes topdown / relu")
        relu_gate = _f32c(relu_gate)
        if relu_gate.shape != y.shape:
            raise ValueError(f"relu_gate {tuple(relu_gate.shape)} != output {tuple(y.shape)}")
    if residual is not None and residual.shape != y.shape:
        raise ValueError(f"residual {tuple(residual.shape)} != output {tuple(y.shape)}")
    if math_mode == "split" and Cout <= 64 and not _NARROW_SPLIT:
        math_mode = "f32"
    flags = (1 if relu else 0) | (2 if relu_after_add else 0) | (8 if flip_taps else 0)
    if math_mode == "split":
        flags |= 4
    lib = _C.lib()
    wkey = (N, H, W, Cin, Cout, KH, KW, stride, pb, pe)
    wsb = _CONV_WS.get(wkey)
    if wsb is None:
        wsb = _CONV_WS[wkey] = lib.d2mi_conv2d_workspace_size(N, H, W, Cin, Cout, KH, KW,
                                                              int(stride), int(pb), int(pe))
    ws = _C.scratch(wsb, x.device) if wsb else None
    st = _C.stream_of(x.device)
    if relu_gate is not None:
        ev = KernelTimer.start()
        rc = lib.d2mi_conv2d_nhwc_gated(_C.ptr(x), _C.ptr(w_packed), _C.ptr(bias),
                                        _C.ptr(residual), _C.ptr(relu_gate), _C.ptr(y), N,
                                        H, W, Cin, Cout, KH, KW, int(stride), int(pb),
                                        int(pe), flags, _C.ptr(ws), wsb, st)
    else:
        ev = KernelTimer.start()
        rc = lib.d2mi_conv2d_nhwc_ex(_C.ptr(x), _C.ptr(w_packed), _C.ptr(bias),
                                     _C.ptr(topdown), _C.ptr(residual), _C.ptr(y), N, H, W,
                                     Cin, Cout, KH, KW, int(stride), int(pb), int(pe), flags,
                                     _C.ptr(ws), wsb, st)
    fl = 2.0 * N * OH * OW * Cout * KH * KW * Cin
    group = "conv2d_split" if math_mode == "split" else "conv2d_mfma"
    KernelTimer.stop(ev, group, fl)
    if ev is not None:
        # the launch's own roofline: its least HBM traffic (every operand read
        # once, the output written once) against its flops, classified at the
        # split ridge (416.7 TF/s / 8 TB/s = 52 flop/B) -- verdict r4: the
        # short-K 1x1s are memory-bound launches, not low-MFMA ones
        byts = conv_bytes(x, w_packed, y, bias, topdown, residual, relu_gate)
        KernelTimer.stop(ev, f"{group}_{bound_of(fl, byts, math_mode)}_bound", fl,
                         extra=lambda: {"bytes": byts})
    if KernelTimer.detail and ev is not None:
        tag = ("g" if relu_gate is not None else "") + ("r" if residual is not None else "") + (
            "f" if flip_taps else "")
        KernelTimer.stop(ev, f"conv {N}x{H}x{W}x{Cin}->{Cout} k{KH} s{stride} p{pb}{pe} {tag}", fl,
                         extra=lambda: {"bytes": byts})
    _C.check(rc, "d2mi_conv2d_nhwc")
    return y


# ridge points of the two product forms: peak flops / HBM bandwidth
SPLIT_RIDGE = 2.5e15 / 6 / 8e12     # 52.1 flop/B (bf16 dense / 6 products)
F32_RIDGE = 157.3e12 / 8e12          # 19.7 flop/B (FP32 matrix)


def conv_bytes(x, w_packed, y, bias=None, topdown=None, residual=None, gate=None):
    """Least HBM bytes of one conv launch: every operand read once, the output
    written once."""
    n = x.numel() + w_packed.numel() + y.numel()
    for t in (bias, topdown, residual, gate):
        if t is not None:
            n += t.numel()
    return 4.0 * n


def bound_of(flops, byts, math_mode="split"):
    ridge = SPLIT_RIDGE if math_mode == "split" else F32_RIDGE
    return "mfma" if flops >= ridge * byts else "hbm"


def conv2d_nhwc_levels(xs, w_packed, bias=None, stride=1, pad=(0, 0), relu=False, math_mode=None):
    """One launch of the same conv over up to 6 feature levels (a head shared
    across FPN levels: RetinaNet / SOLOv2 towers): xs[l] [N_l, H_l, W_l, Cin]
    -> [N_l, OH_l, OW_l, Cout] each (d2mi_conv2d_nhwc_levels).  Every level's
    tiles run in one grid, so the small levels neither serialise behind the
    big one nor need split-K; per-tile arithmetic is conv2d_nhwc's."""
    math_mode = math_mode or CONV_MATH
    if math_mode not in ("f32", "split"):
        raise ValueError(f"conv math must be 'f32' or 'split', got {math_mode!r}")
    xs = [_f32c(x) for x in xs]
    _C.require_device(w_packed, *xs)
    if not 1 <= len(xs) <= 6:
        raise ValueError(f"conv2d_nhwc_levels takes 1..6 levels, got {len(xs)}")
    KH, KW, Cout, Cin = w_packed.shape
    pb, pe = pad
    ys, dims = [], []
    for x in xs:
        N, H, W, C = x.shape
        if C != Cin:
            raise ValueError(f"conv input has {C} channels, weights expect {Cin}")
        OH = (H + pb + pe - KH) // stride + 1
        OW = (W + pb + pe - KW) // stride + 1
        ys.append(torch.empty((N, OH, OW, Cout), dtype=torch.float32, device=x.device))
        dims += [N, H, W]
    if math_mode == "split" and Cout <= 64 and not _NARROW_SPLIT:
        math_mode = "f32"
    flags = (1 if relu else 0) | (4 if math_mode == "split" else 0)
    xp = _C.host_array(_C.c_void_p, [x.data_ptr() for x in xs])
    yp = _C.host_array(_C.c_void_p, [y.data_ptr() for y in ys])
    dm = _C.host_array(_C.ctypes.c_int32, dims)
    lib = _C.lib()
    wsb = lib.d2mi_conv2d_levels_workspace_size(dm, len(xs), Cin, Cout, KH, KW, int(stride),
                                                int(pb), int(pe))
    ws = _C.scratch(wsb, xs[0].device) if wsb else None
    ev = KernelTimer.start()
    rc = lib.d2mi_conv2d_nhwc_levels(xp, dm, len(xs), _C.ptr(w_packed), _C.ptr(bias), yp, Cin,
                                     Cout, KH, KW, int(stride), int(pb), int(pe), flags,
                                     _C.ptr(ws), wsb, _C.stream_of(xs[0].device))
    fl = sum(2.0 * y.shape[0] * y.shape[1] * y.shape[2] * Cout * KH * KW * Cin for y in ys)
    KernelTimer.stop(ev, "conv2d_split" if math_mode == "split" else "conv2d_mfma", fl)
    _C.check(rc, "d2mi_conv2d_nhwc_levels")
    return ys


def conv2d_wgrad(x, dy, kernel_size, stride=1, pad=(0, 0), with_bias=False, math_mode=None,
                 accumulate_into=None):
    """HWIO weight gradient of conv2d_nhwc on the MFMA wgrad kernel; with_bias
    also returns the bias gradient (dy summed over pixels) from the same pass.
    math_mode: "f32" | "split" (None: CONV_MATH), as conv2d_nhwc.
    accumulate_into: the (dw, db) -- or dw -- of an earlier call to add this
    one's gradient into (d2mi_conv2d_wgrad_ex bit 3: old + new in the reduce
    pass, autograd's order for a weight shared by several calls)."""
    math_mode = math_mode or CONV_MATH
    if math_mode not in ("f32", "split"):
        raise ValueError(f"conv math must be 'f32' or 'split', got {math_mode!r}")
    x, dy = _f32c(x), _f32c(dy)
    _C.require_device(x, dy)
    N, H, W, Cin = x.shape
    Cout = dy.shape[-1]
    KH = KW = int(kernel_size)
    pb, pe = pad
    if accumulate_into is not None:
        dw, db = accumulate_into if with_bias else (accumulate_into, None)
        if (dw.shape != (KH, KW, Cin, Cout) or dw.dtype != torch.float32
                or not dw.is_contiguous() or (with_bias and (db is None or db.shape != (Cout,)))):
            raise ValueError("accumulate_into must be the (dw, db) of a wgrad of this shape")
    else:
        dw = torch.empty((KH, KW, Cin, Cout), dtype=torch.float32, device=x.device)
        db = torch.empty((Cout,), dtype=torch.float32, device=x.device) if with_bias else None
    args = (N, H, W, Cin, Cout, KH, KW, int(stride), int(pb), int(pe))
    wsb = _WGRAD_WS.get(args)
    if wsb is None:
        wsb = _WGRAD_WS[args] = _C.lib().d2mi_conv2d_wgrad_workspace_size(*args)
    if accumulate_into is not None:  # (the reduce pass adds: one slab at least)
        wsb = max(wsb, (KH * KW * Cin * Cout + Cout) * 4)
    ws = _C.scratch(wsb, x.device) if wsb else None
    ev = KernelTimer.start()
    flags = (4 if math_mode == "split" else 0) | (8 if accumulate_into is not None else 0)
    rc = _C.lib().d2mi_conv2d_wgrad_ex(_C.ptr(x), _C.ptr(dy), _C.ptr(dw), _C.ptr(db), *args,
                                       flags, _C.ptr(ws), wsb, _C.stream_of(x.device))
    fl = 2.0 * dy.numel() * KH * KW * Cin
    group = "conv2d_wgrad_split" if flags & 4 else "conv2d_wgrad_mfma"
    KernelTimer.stop(ev, group, fl)
    if ev is not None:
        # x and dy read once, dw (+ db) written once (+ read when accumulating)
        byts = 4.0 * (x.numel() + dy.numel() + dw.numel() * (2 if accumulate_into is not None else 1)
                      + (Cout if with_bias else 0))
        KernelTimer.stop(ev, f"{group}_{bound_of(fl, byts, math_mode)}_bound", fl,
                         extra=lambda: {"bytes": byts})
    if KernelTimer.detail and ev is not None:
        KernelTimer.stop(ev, f"wgrad {N}x{H}x{W}x{Cin}->{Cout} k{KH} s{stride}", fl,
                         extra=lambda: {"bytes": byts})
    _C.check(rc, "d2mi_conv2d_wgrad")
    return (dw, db) if with_bias else dw


# ---------------------------------------------------------- FrozenBN fold
class _FoldFrozenBNFn(torch.autograd.Function):
    """(w_eff, b_eff, packed) = conv weights with a frozen BatchNorm folded in
    (d2mi_fold_frozen_bn); packed is the MFMA layout of w_eff (no gradient)."""

    @staticmethod
    def forward(ctx, w, bias, gamma, beta, mean, var, eps, want_packed):
        _C.require_device(w, mean, var)
        KH, KW, Cin, Cout = w.shape
        w = _f32c(w)
        w_eff = torch.empty_like(w)
        packed = (torch.empty((KH, KW, Cout, Cin), dtype=torch.float32, device=w.device)
                  if want_packed else None)
        b_eff = torch.empty((Cout,), dtype=torch.float32, device=w.device)
        rc = _C.lib().d2mi_fold_frozen_bn(_C.ptr(w), _C.ptr(bias), _C.ptr(gamma), _C.ptr(beta),
                                          _C.ptr(mean), _C.ptr(var), float(eps), KH, KW, Cin,
                                          Cout, _C.ptr(w_eff), _C.ptr(packed), _C.ptr(b_eff),
                                          _C.stream_of(w.device))
        _C.check(rc, "d2mi_fold_frozen_bn")
        ctx.save_for_backward(w, bias, gamma, mean, var)
        # packed never gets a gradient: no zero tensor materialised for it
        ctx.set_materialize_grads(False)
        ctx.eps = float(eps)
        ctx.has = (bias is not None, gamma is not None, beta is not None)
        if packed is not None:
            ctx.mark_non_differentiable(packed)
        return w_eff, b_eff, packed

    @staticmethod
    def backward(ctx, gw_eff, gb_eff, _gpacked):
        w, bias, gamma, mean, var = ctx.saved_tensors
        KH, KW, Cin, Cout = w.shape
        has_bias, has_gamma, has_beta = ctx.has
        need = ctx.needs_input_grad
        dev = w.device
        if gw_eff is None:
            gw_eff = torch.zeros_like(w)
        gw_eff = _f32c(gw_eff)
        gb_eff = _f32c(gb_eff) if gb_eff is not None else None
        mk = lambda cond, shape: torch.empty(shape, dtype=torch.float32, device=dev) if cond else None
        gw = mk(need[0], w.shape)
        gbias = mk(has_bias and need[1], (Cout,))
        ggamma = mk(has_gamma and need[2], (Cout,))
        gbeta = mk(has_beta and need[3], (Cout,))
        wsb = _C.lib().d2mi_fold_frozen_bn_bwd_workspace_size(Cout)
        ws = _C.workspace(wsb, dev)
        rc = _C.lib().d2mi_fold_frozen_bn_bwd(
            _C.ptr(gw_eff), _C.ptr(gb_eff), _C.ptr(w), _C.ptr(bias), _C.ptr(gamma), _C.ptr(mean),
            _C.ptr(var), ctx.eps, KH, KW, Cin, Cout, _C.ptr(gw), _C.ptr(gbias), _C.ptr(ggamma),
            _C.ptr(gbeta), _C.ptr(ws), wsb, _C.stream_of(dev))
        _C.check(rc, "d2mi_fold_frozen_bn_bwd")
        return gw, gbias, ggamma, gbeta, None, None, None, None


def fold_frozen_bn(w_hwio, bias, gamma, beta, mean, var, eps, want_packed=False):
    """Conv weights (HWIO) with a frozen BatchNorm folded in: returns
    (w_eff, b_eff, packed-or-None), differentiable w.r.t. w, bias, gamma, beta."""
    return _FoldFrozenBNFn.apply(w_hwio, bias, gamma, beta, mean, var, float(eps),
                                 bool(want_packed))


def match_boxes(gt_boxes, gt_flags, boxes, thresholds, labels_of, allow_low_quality,
                crowd_thr=1e-3, difficult_thr=float("inf")):
    """Fused pairwise IoU + Matcher (d2mi_match_boxes): gt_boxes [N, G, 4],
    gt_flags [N, G] int (bit0 matchable, bit1 crowd, bit2 difficult), boxes
    [P, 4] (shared) or [N, P, 4]; thresholds with the -inf / +inf ends.
    Returns (matches int64 [N, P], labels int64 [N, P])."""
    gt_boxes = _f32c(gt_boxes)
    boxes = _f32c(boxes)
    gt_flags = _i32c(gt_flags)
    _C.require_device(gt_boxes, gt_flags, boxes)
    N, G = gt_flags.shape
    per_image = boxes.dim() == 3
    P = boxes.shape[-2]
    matches = torch.empty((N, P), dtype=torch.int64, device=boxes.device)
    labels = torch.empty((N, P), dtype=torch.int64, device=boxes.device)
    thr = _C.host_array(_C.c_float, [float(t) for t in thresholds])
    lab = _C.host_array(_C.ctypes.c_int32, [int(v) for v in labels_of])
    wsb = _C.lib().d2mi_match_workspace_size(N, G)
    ws = _C.workspace(wsb, boxes.device)
    rc = _C.lib().d2mi_match_boxes(_C.ptr(gt_boxes), _C.ptr(gt_flags), _C.ptr(boxes),
                                   int(per_image), N, G, P, thr, lab, len(labels_of),
                                   int(bool(allow_low_quality)), float(crowd_thr),
                                   float(difficult_thr), _C.ptr(matches), _C.ptr(labels),
                                   _C.ptr(ws), wsb, _C.stream_of(boxes.device))
    _C.check(rc, "d2mi_match_boxes")
    return matches, labels


def _mask_u8(m):
    """A [N, G] bool / integer mask as contiguous bytes (bool: a free view)."""
    if m is None:
        return None
    m = m.contiguous()
    return m.view(torch.uint8) if m.dtype == torch.bool else (m != 0).view(torch.uint8)


def match_boxes_masks(gt_boxes, valid, boxes, thresholds, labels_of, allow_low_quality,
                      crowd=None, difficult=None, crowd_thr=1e-3, difficult_thr=float("inf")):
    """match_boxes with the GT flags as [N, G] masks (d2mi_match_boxes_ex):
    valid required, crowd / difficult optional -- the bool tensors are passed
    as they are, no int32 packing launches; the matchable GT are valid and
    neither crowd nor difficult."""
    gt_boxes = _f32c(gt_boxes)
    boxes = _f32c(boxes)
    m, c, d = _mask_u8(valid), _mask_u8(crowd), _mask_u8(difficult)
    _C.require_device(gt_boxes, m, boxes, *[t for t in (c, d) if t is not None])
    N, G = m.shape
    for t in (c, d):
        if t is not None and tuple(t.shape) != (N, G):
            raise ValueError("match_boxes_masks: crowd / difficult must be [N, G] like matchable")
    per_image = boxes.dim() == 3
    P = boxes.shape[-2]
    matches = torch.empty((N, P), dtype=torch.int64, device=boxes.device)
    labels = torch.empty((N, P), dtype=torch.int64, device=boxes.device)
    thr = _C.host_array(_C.c_float, [float(t) for t in thresholds])
    lab = _C.host_array(_C.ctypes.c_int32, [int(v) for v in labels_of])
    wsb = _C.lib().d2mi_match_workspace_size(N, G)
    ws = _C.workspace(wsb, boxes.device)
    nul = _C.c_void_p(None)
    rc = _C.lib().d2mi_match_boxes_ex(_C.ptr(gt_boxes), _C.ptr(m),
                                      _C.ptr(c) if c is not None else nul,
                                      _C.ptr(d) if d is not None else nul, _C.ptr(boxes),
                                      int(per_image), N, G, P, thr, lab, len(labels_of),
                                      int(bool(allow_low_quality)), float(crowd_thr),
                                      float(difficult_thr), _C.ptr(matches), _C.ptr(labels),
                                      _C.ptr(ws), wsb, _C.stream_of(boxes.device))
    _C.check(rc, "d2mi_match_boxes_ex")
    return matches, labels


class _RPNLossFn(torch.autograd.Function):
    """(loss_cls_sum, loss_loc_sum) * scale of the RPN (d2mi_rpn_loss_fwd /
    d2mi_rpn_loss_bwd_ex); differentiable w.r.t. logits and deltas.  The scale
    (the normaliser x loss weight) is applied to the two sums here and to the
    upstream gradients inside the backward kernel: no multiply launches."""

    @staticmethod
    def forward(ctx, logits, deltas, anchors, gt_boxes, matches, pos, sampled, weights, beta,
                scale=1.0):
        N, P = logits.shape
        G = gt_boxes.shape[1]
        nb = _C.lib().d2mi_rpn_loss_blocks()
        part = torch.empty((N * nb, 2), dtype=torch.float32, device=logits.device)
        w = _C.host_array(_C.c_float, [float(v) for v in weights])
        rc = _C.lib().d2mi_rpn_loss_fwd(_C.ptr(logits), _C.ptr(deltas), _C.ptr(anchors),
                                        _C.ptr(gt_boxes), _C.ptr(matches), _C.ptr(pos),
                                        _C.ptr(sampled), N, P, G, w, float(beta), _C.ptr(part),
                                        _C.stream_of(logits.device))
        _C.check(rc, "d2mi_rpn_loss_fwd")
        ctx.save_for_backward(logits, deltas, anchors, gt_boxes, matches, pos, sampled)
        ctx.conf = (tuple(float(v) for v in weights), float(beta), float(scale))
        ctx.set_materialize_grads(False)  # a missing gradient is a zero one (null pointer)
        # fixed-size reduction of the partials (deterministic order), scaled
        out = part.sum(0)
        if scale != 1.0:
            out.mul_(scale)
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_cls, g_loc):
        logits, deltas, anchors, gt_boxes, matches, pos, sampled = ctx.saved_tensors
        weights, beta, scale = ctx.conf
        N, P = logits.shape
        dev = logits.device
        g_cls = _f32c(g_cls) if g_cls is not None else None
        g_loc = _f32c(g_loc) if g_loc is not None else None
        d_logits = torch.empty_like(logits)
        d_deltas = torch.empty_like(deltas)
        w = _C.host_array(_C.c_float, list(weights))
        nul = _C.c_void_p(None)
        rc = _C.lib().d2mi_rpn_loss_bwd_ex(_C.ptr(logits), _C.ptr(deltas), _C.ptr(anchors),
                                           _C.ptr(gt_boxes), _C.ptr(matches), _C.ptr(pos),
                                           _C.ptr(sampled), N, P, gt_boxes.shape[1], w, beta,
                                           _C.ptr(g_cls) if g_cls is not None else nul,
                                           _C.ptr(g_loc) if g_loc is not None else nul,
                                           float(scale), _C.ptr(d_logits), _C.ptr(d_deltas),
                                           _C.stream_of(dev))
        _C.check(rc, "d2mi_rpn_loss_bwd_ex")
        return d_logits, d_deltas, None, None, None, None, None, None, None, None


class _FastRCNNLossFn(torch.autograd.Function):
    """(loss_cls, loss_box_reg) of FastRCNNOutputs.losses on dense rows
    (d2mi_fast_rcnn_loss_fwd / _bwd, csrc/roi_losses.hip); differentiable
    w.r.t. logits and deltas."""

    @staticmethod
    def forward(ctx, logits, deltas, proposals, gt_classes, gt_boxes, valid, weights, beta):
        B, K1 = logits.shape
        nreg = deltas.shape[1] // 4
        dev = logits.device
        stats = torch.empty(4, dtype=torch.float32, device=dev)
        lib = _C.lib()
        wsb = lib.d2mi_fast_rcnn_loss_workspace_size(B)
        ws = _C.scratch(wsb, dev)
        w = _C.host_array(_C.c_float, [float(v) for v in weights])
        rc = lib.d2mi_fast_rcnn_loss_fwd(_C.ptr(logits), _C.ptr(deltas), _C.ptr(proposals),
                                         _C.ptr(gt_classes), _C.ptr(gt_boxes), _C.ptr(valid), B,
                                         K1, nreg, w, float(beta), _C.ptr(stats), _C.ptr(ws), wsb,
                                         _C.stream_of(dev))
        _C.check(rc, "d2mi_fast_rcnn_loss_fwd")
        ctx.save_for_backward(logits, deltas, proposals, gt_classes, gt_boxes, valid, stats)
        ctx.conf = (tuple(float(v) for v in weights), float(beta))
        ctx.set_materialize_grads(False)
        return stats[0], stats[1]

    @staticmethod
    def backward(ctx, g_cls, g_box):
        logits, deltas, proposals, gt_classes, gt_boxes, valid, stats = ctx.saved_tensors
        weights, beta = ctx.conf
        dev = logits.device
        z = torch.zeros((), dtype=torch.float32, device=dev)
        grads = torch.stack([g_cls if g_cls is not None else z,
                             g_box if g_box is not None else z]).float().contiguous()
        d_logits = torch.empty_like(logits)
        d_deltas = torch.empty_like(deltas)
        B, K1 = logits.shape
        w = _C.host_array(_C.c_float, list(weights))
        rc = _C.lib().d2mi_fast_rcnn_loss_bwd(_C.ptr(logits), _C.ptr(deltas), _C.ptr(proposals),
                                              _C.ptr(gt_classes), _C.ptr(gt_boxes), _C.ptr(valid),
                                              B, K1, deltas.shape[1] // 4, w, beta, _C.ptr(stats),
                                              _C.ptr(grads), _C.ptr(d_logits), _C.ptr(d_deltas),
                                              _C.stream_of(dev))
        _C.check(rc, "d2mi_fast_rcnn_loss_bwd")
        return d_logits, d_deltas, None, None, None, None, None, None


def fast_rcnn_loss(logits, deltas, proposals, gt_classes, gt_boxes, valid, weights, beta):
    """Fused Fast R-CNN losses on dense rows: logits [B, K+1], deltas
    [B, nreg*4], proposals / gt_boxes [B, 4], gt_classes [B], valid [B] ->
    (loss_cls, loss_box_reg), both already / max(1, #valid)."""
    logits, deltas = _f32c(logits), _f32c(deltas)
    proposals, gt_boxes = _f32c(proposals), _f32c(gt_boxes)
    gt_classes = gt_classes.to(torch.int64).contiguous()
    valid = valid.to(torch.uint8).contiguous()
    _C.require_device(logits, deltas, proposals, gt_classes, gt_boxes, valid)
    return _FastRCNNLossFn.apply(logits, deltas, proposals, gt_classes, gt_boxes, valid,
                                 tuple(weights), float(beta))


class _MaskLossFn(torch.autograd.Function):
    """mask_rcnn_loss's sigmoid BCE of the gt-class channel over foreground
    rows, mean over fg x Hm x Wm (d2mi_mask_loss_fwd / _bwd)."""

    @staticmethod
    def forward(ctx, logits, target, classes, fg):
        B, Hm, Wm, C = logits.shape
        dev = logits.device
        stats = torch.empty(3, dtype=torch.float32, device=dev)
        lib = _C.lib()
        wsb = lib.d2mi_mask_loss_workspace_size(B)
        ws = _C.scratch(wsb, dev)
        rc = lib.d2mi_mask_loss_fwd(_C.ptr(logits), _C.ptr(target), _C.ptr(classes), _C.ptr(fg), B,
                                    Hm * Wm, C, _C.ptr(stats), _C.ptr(ws), wsb, _C.stream_of(dev))
        _C.check(rc, "d2mi_mask_loss_fwd")
        ctx.save_for_backward(logits, target, classes, fg, stats)
        return stats[0]

    @staticmethod
    def backward(ctx, g):
        logits, target, classes, fg, stats = ctx.saved_tensors
        B, Hm, Wm, C = logits.shape
        grads = g.reshape(1).float().contiguous()
        d_logits = torch.empty_like(logits)
        rc = _C.lib().d2mi_mask_loss_bwd(_C.ptr(logits), _C.ptr(target), _C.ptr(classes),
                                         _C.ptr(fg), B, Hm * Wm, C, _C.ptr(stats), _C.ptr(grads),
                                         _C.ptr(d_logits), _C.stream_of(logits.device))
        _C.check(rc, "d2mi_mask_loss_bwd")
        return d_logits, None, None, None


def mask_loss(logits, target, classes, fg):
    """Fused mask loss: logits [B, Hm, Wm, C], target [B, Hm, Wm] (0 / 1),
    classes [B], fg [B] -> mean sigmoid BCE of each fg row's class channel."""
    logits, target = _f32c(logits), _f32c(target)
    classes = classes.to(torch.int64).contiguous()
    fg = fg.to(torch.uint8).contiguous()
    _C.require_device(logits, target, classes, fg)
    return _MaskLossFn.apply(logits, target, classes, fg)


def rpn_loss(logits, deltas, anchors, gt_boxes, matches, pos, sampled, weights, beta,
             scale=1.0):
    """Fused RPN losses: logits [N, P], deltas [N, P, 4], anchors [P, 4],
    gt_boxes [N, G, 4], matches [N, P], pos / sampled [N, P] bool ->
    (loss_cls_sum * scale, loss_loc_sum * scale); scale = the caller's
    normaliser (1.0: the plain sums)."""
    logits, deltas = _f32c(logits), _f32c(deltas)
    anchors, gt_boxes = _f32c(anchors), _f32c(gt_boxes)
    matches = matches.to(torch.int64).contiguous()
    pos, sampled = _mask_u8(pos), _mask_u8(sampled)
    _C.require_device(logits, deltas, anchors, gt_boxes, matches, pos, sampled)
    return _RPNLossFn.apply(logits, deltas, anchors, gt_boxes, matches, pos, sampled,
                            tuple(weights), float(beta), float(scale))


class _RetinaLossFn(torch.autograd.Function):
    """(focal loss sum, smooth-L1 sum) of RetinaNet.losses over the head's
    per-level outputs (d2mi_retina_loss_fwd / _bwd, csrc/retina_loss.hip);
    differentiable w.r.t. every level's class logits and box deltas."""

    @staticmethod
    def forward(ctx, conf, anchors, gt_boxes, gt_classes, matches, labels, *levels):
        L = len(levels) // 2
        cls, box = levels[:L], levels[L:]
        N, K, A = cls[0].shape[0], conf[0], conf[1]
        lvl = [int(c.shape[1] * c.shape[2] * A) for c in cls]
        nb = _C.lib().d2mi_retina_loss_blocks()
        dev = anchors.device
        part = torch.empty((N * nb, 2), dtype=torch.float32, device=dev)
        la = _C.host_array(_C.ctypes.c_longlong, lvl)
        w = _C.host_array(_C.c_float, list(conf[5]))
        cp = _C.host_array(_C.c_void_p, [c.data_ptr() for c in cls])
        bp = _C.host_array(_C.c_void_p, [b.data_ptr() for b in box])
        rc = _C.lib().d2mi_retina_loss_fwd(cp, bp, la, L, N, K, A, _C.ptr(anchors),
                                           _C.ptr(gt_boxes), _C.ptr(gt_classes),
                                           gt_boxes.shape[1], _C.ptr(matches), _C.ptr(labels),
                                           conf[2], conf[3], conf[4], w, _C.ptr(part),
                                           _C.stream_of(dev))
        _C.check(rc, "d2mi_retina_loss_fwd")
        ctx.save_for_backward(anchors, gt_boxes, gt_classes, matches, labels, *levels)
        ctx.conf = (conf, lvl)
        ctx.set_materialize_grads(False)  # a missing gradient is a zero one (null pointer)
        out = part.sum(0)  # fixed-size reduction of the partials: deterministic order
        return out[0], out[1]

    @staticmethod
    def backward(ctx, g_cls, g_box):
        anchors, gt_boxes, gt_classes, matches, labels, *levels = ctx.saved_tensors
        conf, lvl = ctx.conf
        L = len(levels) // 2
        cls, box = levels[:L], levels[L:]
        N, K, A = cls[0].shape[0], conf[0], conf[1]
        d = [torch.empty_like(t) for t in levels]
        nul = _C.c_void_p(None)
        g_cls = _f32c(g_cls) if g_cls is not None else None
        g_box = _f32c(g_box) if g_box is not None else None
        rc = _C.lib().d2mi_retina_loss_bwd(
            _C.host_array(_C.c_void_p, [c.data_ptr() for c in cls]),
            _C.host_array(_C.c_void_p, [b.data_ptr() for b in box]),
            _C.host_array(_C.c_void_p, [t.data_ptr() for t in d[:L]]),
            _C.host_array(_C.c_void_p, [t.data_ptr() for t in d[L:]]),
            _C.host_array(_C.ctypes.c_longlong, lvl), L, N, K, A, _C.ptr(anchors),
            _C.ptr(gt_boxes), _C.ptr(gt_classes), gt_boxes.shape[1], _C.ptr(matches),
            _C.ptr(labels), conf[2], conf[3], conf[4], _C.host_array(_C.c_float, list(conf[5])),
            _C.ptr(g_cls) if g_cls is not None else nul,
            _C.ptr(g_box) if g_box is not None else nul, _C.stream_of(anchors.device))
        _C.check(rc, "d2mi_retina_loss_bwd")
        return (None,) * 6 + tuple(d)


def retina_loss(cls_levels, box_levels, anchors, gt_boxes, gt_classes, matches, labels,
                num_classes, num_anchors, alpha, gamma, beta, weights):
    """Fused RetinaNet losses (retinanet.py:147-210, before the normaliser):
    cls_levels [N, H, W, A*K] / box_levels [N, H, W, A*4] per level, anchors
    [R, 4] (levels concatenated, (h, w, a) order), gt_boxes [N, G, 4],
    gt_classes [N, G], matches / labels [N, R] (the Matcher's; labels 1 fg,
    0 bg, -1 ignore) -> (sum of sigmoid_focal_loss over every valid anchor and
    class, sum of smooth_l1 over the foreground anchors' deltas)."""
    cls_levels = [_f32c(c) for c in cls_levels]
    box_levels = [_f32c(b) for b in box_levels]
    anchors, gt_boxes = _f32c(anchors), _f32c(gt_boxes)
    gt_classes = gt_classes.to(torch.int64).contiguous()
    matches = matches.to(torch.int64).contiguous()
    labels = labels.to(torch.int64).contiguous()
    _C.require_device(anchors, gt_boxes, gt_classes, matches, labels, *cls_levels, *box_levels)
    for c, b in zip(cls_levels, box_levels):
        if c.shape[-1] != num_anchors * num_classes or b.shape[-1] != num_anchors * 4 \
                or c.shape[:3] != b.shape[:3]:
            raise ValueError(f"retina loss: level outputs {tuple(c.shape)} / {tuple(b.shape)} do "
                             f"not match A={num_anchors}, K={num_classes}")
    R = sum(int(c.shape[1] * c.shape[2]) * num_anchors for c in cls_levels)
    if anchors.shape[0] != R or labels.shape[-1] != R:
        raise ValueError(f"retina loss: {anchors.shape[0]} anchors / {labels.shape[-1]} labels "
                         f"for {R} head outputs")
    conf = (int(num_classes), int(num_anchors), float(alpha), float(gamma), float(beta),
            tuple(float(v) for v in weights))
    return _RetinaLossFn.apply(conf, anchors, gt_boxes, gt_classes, matches, labels,
                               *cls_levels, *box_levels)


def stem_conv_weights(w):
    """HWIO [7, 7, 3, Cout=64] -> the [3][64][160] bf16 planes d2mi_stem_conv
    takes (K = (kh * 7 + kw) * 3 + c, zero-padded to 160)."""
    if tuple(w.shape) != (7, 7, 3, 64):
        raise ValueError(f"stem conv weights must be [7, 7, 3, 64], got {tuple(w.shape)}")
    wt = torch.zeros((64, 160), dtype=torch.float32, device=w.device)
    wt[:, :147] = _f32c(w).reshape(147, 64).t()
    return split_bf16x3(wt.contiguous())


def stem_conv(x, w3):
    """d2mi_stem_conv: the 7x7 / stride-2 stem conv (Cin 3 -> 64, pad 3) on
    the split-bf16 MFMA; x [N, H, W, 3] NHWC, w3 from stem_conv_weights.
    Raw sums (the folded shift is stem_pool's); no gradient."""
    x = _f32c(x)
    _C.require_device(x, w3)
    N, H, W, C = x.shape
    if C != 3:
        raise ValueError(f"stem conv takes 3 input channels, got {C}")
    y = torch.empty((N, (H - 1) // 2 + 1, (W - 1) // 2 + 1, 64), dtype=torch.float32,
                    device=x.device)
    rc = _C.lib().d2mi_stem_conv(_C.ptr(x), _C.ptr(w3), N, H, W, _C.ptr(y),
                                 _C.stream_of(x.device))
    _C.check(rc, "d2mi_stem_conv")
    return y


# Device images preprocessed by d2mi_preprocess_images (False: torch's
# subtract / divide / flip / pad, five launches; tests compare;
# D2MI_FUSED_PREPROCESS=0 for a bench A/B).
FUSED_PREPROCESS = os.environ.get("D2MI_FUSED_PREPROCESS", "1") != "0"


def preprocess_images(x, mean, std, flip, size_divisibility=0):
    """d2mi_preprocess_images: (x - mean) / std, the BGR channel flip and the
    zero pad to size_divisibility in one pass (rcnn.py:146-157 +
    image_list.py:89-100); x [N, H, W, 3] NHWC f32 -> [N, Hp, Wp, 3]."""
    x = _f32c(x)
    mean, std = _f32c(mean), _f32c(std)
    _C.require_device(x, mean, std)
    N, H, W, C = x.shape
    if C != 3 or mean.numel() != 3 or std.numel() != 3:
        raise ValueError(f"preprocess takes 3 channels and 3 means / stds, got {tuple(x.shape)}")
    s = int(size_divisibility)
    Hp, Wp = (H + (-H) % s, W + (-W) % s) if s > 0 else (H, W)
    out = torch.empty((N, Hp, Wp, 3), dtype=torch.float32, device=x.device)
    rc = _C.lib().d2mi_preprocess_images(_C.ptr(x), _C.ptr(mean), _C.ptr(std), N, H, W, Hp, Wp,
                                         int(bool(flip)), _C.ptr(out), _C.stream_of(x.device))
    _C.check(rc, "d2mi_preprocess_images")
    return out


def stem_pool(y, shift=None):
    """relu(y + shift) -> zero pad 1 -> 3x3 / 2 VALID max pool, NHWC
    (d2mi_stem_pool): the ResNet stem tail in one pass (no gradient)."""
    y = _f32c(y)
    shift = _f32c(shift) if shift is not None else None
    _C.require_device(y)
    N, H, W, C = y.shape
    out = torch.empty((N, (H - 1) // 2 + 1, (W - 1) // 2 + 1, C), dtype=torch.float32,
                      device=y.device)
    rc = _C.lib().d2mi_stem_pool(_C.ptr(y), _C.ptr(shift), N, H, W, C, _C.ptr(out),
                                 _C.stream_of(y.device))
    _C.check(rc, "d2mi_stem_pool")
    return out


def upsample2x_grad(gy):
    """Adjoint of the FPN top-down nearest 2x upsample (d2mi_upsample2x_grad):
    gy [N, OH, OW, C] -> [N, ceil(OH/2), ceil(OW/2), C]."""
    gy = _f32c(gy)
    _C.require_device(gy)
    N, OH, OW, C = gy.shape
    out = torch.empty((N, (OH + 1) // 2, (OW + 1) // 2, C), dtype=torch.float32, device=gy.device)
    rc = _C.lib().d2mi_upsample2x_grad(_C.ptr(gy), N, OH, OW, C, _C.ptr(out),
                                       _C.stream_of(gy.device))
    _C.check(rc, "d2mi_upsample2x_grad")
    return out


def stride_scatter(g, out_shape, stride, add=None, add2=None, gate=None):
    """Input gradient of a 1x1 stride-s conv from its GEMM on the strided grid
    (d2mi_stride_scatter_ex): zeros off the grid, + add, + add2 (nullable, in
    that order), then zeroed where gate <= 0 (gate nullable: the ReLU backward
    of the ReLU output ``gate``)."""
    g = _f32c(g)
    add = _f32c(add) if add is not None else None
    add2 = _f32c(add2) if add2 is not None else None
    gate = _f32c(gate) if gate is not None else None
    _C.require_device(g)
    N, H, W, C = out_shape
    if g.shape != (N, (H - 1) // stride + 1, (W - 1) // stride + 1, C):
        raise ValueError(f"stride_scatter: {tuple(g.shape)} is not the stride-{stride} grid of "
                         f"{tuple(out_shape)}")
    for t in (add, add2, gate):
        if t is not None and tuple(t.shape) != tuple(out_shape):
            raise ValueError(f"stride_scatter: operand {tuple(t.shape)} != {tuple(out_shape)}")
    out = torch.empty(tuple(out_shape), dtype=torch.float32, device=g.device)
    rc = _C.lib().d2mi_stride_scatter_ex(_C.ptr(g), _C.ptr(add), _C.ptr(add2), _C.ptr(gate), N, H,
                                         W, C, int(stride), _C.ptr(out), _C.stream_of(g.device))
    _C.check(rc, "d2mi_stride_scatter_ex")
    return out


_FOLD_DT = np.dtype([(n, np.uint64) for n in (
    "w", "bias", "gamma", "beta", "mean", "var", "w_eff", "w_packed", "b_eff", "gw_eff", "gb_eff",
    "gw", "gbias", "ggamma", "gbeta")] + [("eps", np.float32)] + [(n, np.int32) for n in (
        "taps", "Cin", "Cout", "fwd_begin", "bwd_begin", "co_begin", "pad")] + [
    ("partial_offset", np.int64)])


class _HostTable:
    """A device copy of a host table uploaded through a small ring of pinned
    buffers (each slot reused once its previous copy has left, by event)."""
    RING = 4

    def __init__(self, nbytes, device, what="table"):
        self.what = what
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
        self.ring = [torch.empty(nbytes, dtype=torch.uint8).pin_memory() for _ in range(self.RING)]
        self.events = [None] * self.RING
        self.i = 0

    def upload(self, arr):
        if capture.capturing():  # a per-graph table, filled after the capture
            return capture.table(arr, self.dev.device, self.what)
        k = self.i
        self.i = (k + 1) % self.RING
        if self.events[k] is not None:
            self.events[k].synchronize()
        self.ring[k].numpy()[:] = arr.view(np.uint8)
        self.dev.copy_(self.ring[k], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev.device))
        self.events[k] = ev
        return self.dev


_fold_tables = {}


def _fold_table(kind, n, device):
    key = (kind, n, device)
    t = _fold_tables.get(key)
    if t is None:
        sz, chunks = _C.ctypes.c_int(), _C.ctypes.c_int()
        _C.lib().d2mi_fold_many_sizes(_C.ctypes.byref(sz), _C.ctypes.byref(chunks))
        if sz.value != _FOLD_DT.itemsize:
            raise RuntimeError("d2mi_fold_entry layout mismatch")
        t = _fold_tables[key] = (_HostTable(n * _FOLD_DT.itemsize, device, f"fold {kind}"),
                                 chunks.value)
    return t


def _addr(t):
    return 0 if t is None else t.data_ptr()


def _sole_owner(t):
    """True when no tensor but ``t`` itself uses t's storage (no live view)."""
    return torch._C._storage_Use_Count(t.untyped_storage()._cdata) <= 2


class _FoldPlan:
    """The forward fold of one set of layers, kept across training steps: the
    parameters are updated in place (same addresses every step), so the
    entry table and the three flat output buffers are reused -- one launch
    over a table already on the device, no host table rebuild or upload --
    whenever none of last step's output views is still alive (the previous
    step's graph is gone)."""

    def __init__(self, flats, tab, fwd, shapes, dev):
        self.flats, self.tab, self.fwd, self.shapes = flats, tab, fwd, shapes
        self.dev_tab = torch.empty(tab.nbytes, dtype=torch.uint8, device=dev)
        self.dev_tab.copy_(torch.from_numpy(tab.view(np.uint8)))

    def reusable(self):
        return all(_sole_owner(f) for f in self.flats)

    def views(self):
        sizes, couts, psz, shapes = self.shapes
        w_effs = self.flats[0].split(sizes)
        b_effs = self.flats[1].split(couts)
        packs = self.flats[2].split(psz)
        outs = []
        for i, (KH, KW, Cin, Cout) in enumerate(shapes):
            outs += [w_effs[i].view(KH, KW, Cin, Cout), b_effs[i],
                     packs[i].view(KH, KW, Cout, Cin) if psz[i] else None]
        return outs


_fold_plans = {}


class _FoldManyFn(torch.autograd.Function):
    """Every BN-conv of the network folded at once: d2mi_fold_frozen_bn_many
    (one launch) forward, d2mi_fold_frozen_bn_bwd_many (two launches)
    backward.  inputs: per entry (w, bias, gamma, beta, mean, var); outputs:
    per entry (w_eff, b_eff, packed-or-None).  Repeated folds of the same
    parameters run from a _FoldPlan."""

    @staticmethod
    def forward(ctx, spec, *ts):
        n = len(spec)
        dev = ts[0].device
        key = (spec, dev, tuple(_addr(t) for t in ts), tuple(ts[6 * i].shape for i in range(n)))
        plan = None if capture.capturing() else _fold_plans.get(key)
        if plan is not None and plan.reusable():
            outs = plan.views()
            for i in range(n):
                if outs[3 * i + 2] is not None:
                    ctx.mark_non_differentiable(outs[3 * i + 2])
            rc = _C.lib().d2mi_fold_frozen_bn_many(_C.ptr(plan.dev_tab), n, plan.fwd,
                                                   _C.stream_of(dev))
            _C.check(rc, "d2mi_fold_frozen_bn_many")
            ctx.save_for_backward(*ts)
            ctx.tab, ctx.sizes = plan.tab, plan.bwd_sizes
            ctx.set_materialize_grads(False)
            return tuple(outs)
        rows, outs = [], []
        fwd = bwd = cob = part = 0
        table, chunks = _fold_table("fwd", n, dev)
        ws_ = [ts[6 * i] for i in range(n)]
        for w in ws_:
            if not (w.is_contiguous() and w.dtype == torch.float32 and w.device == dev):
                raise ValueError("fold_frozen_bn_many: contiguous f32 weights on one device")
        # the outputs are views of three flat buffers (3 allocations, not 3n)
        sizes = [w.numel() for w in ws_]
        couts = [w.shape[3] for w in ws_]
        flats = (torch.empty(sum(sizes), dtype=torch.float32, device=dev),
                 torch.empty(sum(couts), dtype=torch.float32, device=dev),
                 torch.empty(max(sum(sz if sp[1] else 0 for sz, sp in zip(sizes, spec)), 1),
                             dtype=torch.float32, device=dev))
        w_effs = flats[0].split(sizes)
        b_effs = flats[1].split(couts)
        psz = [sz if sp[1] else 0 for sz, sp in zip(sizes, spec)]
        packs = flats[2].split(psz)
        for i, (eps, want_packed) in enumerate(spec):
            w, bias, gamma, beta, mean, var = ts[6 * i:6 * i + 6]
            KH, KW, Cin, Cout = w.shape
            w_eff = w_effs[i].view(KH, KW, Cin, Cout)
            b_eff = b_effs[i]
            packed = packs[i].view(KH, KW, Cout, Cin) if want_packed else None
            nco, taps = -(-Cout // 64), KH * KW
            rows.append((_addr(w), _addr(bias), _addr(gamma), _addr(beta),
                         _addr(mean), _addr(var), _addr(w_eff), _addr(packed), _addr(b_eff),
                         0, 0, 0, 0, 0, 0, eps, taps, Cin, Cout, fwd, bwd, cob, 0, part))
            fwd += nco * -(-Cin // 64) * taps
            bwd += nco * chunks
            cob += Cout
            part += chunks * Cout
            outs += [w_eff, b_eff, packed]
            if packed is not None:
                ctx.mark_non_differentiable(packed)
        tab = np.array(rows, dtype=_FOLD_DT)
        rc = _C.lib().d2mi_fold_frozen_bn_many(_C.ptr(table.upload(tab)), n, fwd,
                                               _C.stream_of(dev))
        _C.check(rc, "d2mi_fold_frozen_bn_many")
        if not capture.capturing():
            if len(_fold_plans) > 4:  # (each holds its outputs: ~0.2 GB for R50)
                _fold_plans.clear()
            plan = _FoldPlan(flats, tab.copy(), fwd,
                             (sizes, couts, psz, [tuple(w.shape) for w in ws_]), dev)
            plan.bwd_sizes = (bwd, cob, part)
            _fold_plans[key] = plan
        ctx.save_for_backward(*ts)
        ctx.tab, ctx.sizes = tab, (bwd, cob, part)
        ctx.set_materialize_grads(False)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        ts = ctx.saved_tensors
        tab = ctx.tab
        n = len(tab)
        need = ctx.needs_input_grad[1:]
        dev = ts[0].device
        bwd, cob, part = ctx.sizes
        ret = [None]
        keep = []
        cols = [[0] * n for _ in range(6)]  # gw_eff gb_eff gw gbias ggamma gbeta
        for i in range(n):
            w, bias, gamma, beta = ts[6 * i:6 * i + 4]
            gw_eff, gb_eff = grads[3 * i], grads[3 * i + 1]
            if gw_eff is not None:
                gw_eff = _f32c(gw_eff)
            if gb_eff is not None:
                gb_eff = _f32c(gb_eff)
            keep += [gw_eff, gb_eff]
            k = 6 * i
            gw = torch.empty_like(w) if need[k] else None
            gbias = torch.empty_like(bias) if need[k + 1] and bias is not None else None
            ggamma = torch.empty_like(gamma) if need[k + 2] and gamma is not None else None
            gbeta = torch.empty_like(beta) if need[k + 3] and beta is not None else None
            for c, t in enumerate((gw_eff, gb_eff, gw, gbias, ggamma, gbeta)):
                if t is not None:
                    cols[c][i] = t.data_ptr()
            ret += [gw, gbias, ggamma, gbeta, None, None]
        for c, name in enumerate(("gw_eff", "gb_eff", "gw", "gbias", "ggamma", "gbeta")):
            tab[name] = cols[c]
        table, _ = _fold_table("bwd", n, dev)
        ws = _C.scratch(part * 4, dev)
        rc = _C.lib().d2mi_fold_frozen_bn_bwd_many(_C.ptr(table.upload(tab)), n, bwd, cob,
                                                   _C.ptr(ws), _C.stream_of(dev))
        _C.check(rc, "d2mi_fold_frozen_bn_bwd_many")
        del keep
        return tuple(ret)


def fold_frozen_bn_many(entries):
    """entries: [(w_hwio, bias, gamma, beta, mean, var, eps, want_packed)] ->
    [(w_eff, b_eff, packed-or-None)], the batched fold_frozen_bn (bit-identical
    results, differentiable w.r.t. each w, bias, gamma, beta)."""
    if not entries:
        return []
    spec = tuple((float(e[6]), bool(e[7])) for e in entries)
    ts = []
    for e in entries:
        _C.require_device(e[0], e[4], e[5])
        ts += [_f32c(e[0])] + [None if t is None else _f32c(t) for t in e[1:4]] + [
            _f32c(e[4]), _f32c(e[5])]
    outs = _FoldManyFn.apply(spec, *ts)
    return [tuple(outs[3 * i:3 * i + 3]) for i in range(len(entries))]


# -------------------------------------------------------------- matrix NMS
def matrix_nms_scores(masks, classes, scores, sum_masks=None, kernel="gaussian", sigma=2.0):
    if kernel not in ("gaussian", "linear"):
        raise NotImplementedError(f"NMS kernel {kernel} not implemented yet.")
    M = masks.shape[0]
    masks2 = _f32c(masks.reshape(M, -1))
    classes = classes.to(torch.int64).contiguous()
    scores = _f32c(scores)
    _C.require_device(masks2, classes, scores)
    sm = _f32c(sum_masks) if sum_masks is not None else None
    out = torch.empty_like(scores)
    wsb = _C.lib().d2mi_matrix_nms_workspace_size(M)
    ws = _C.workspace(wsb, masks.device)
    rc = _C.lib().d2mi_matrix_nms(_C.ptr(masks2), _C.ptr(classes), _C.ptr(scores), _C.ptr(sm), M,
                                  masks2.shape[1], 0 if kernel == "gaussian" else 1, float(sigma),
                                  _C.ptr(out), _C.ptr(ws), wsb, _C.stream_of(masks.device))
    _C.check(rc, "d2mi_matrix_nms")
    return out


# ---------------------------------------------------------------- GroupNorm
def group_norm(x, num_groups, gamma, beta, eps, relu=False, up2=False, accumulate_into=None):
    """GroupNorm (+ ReLU) on NHWC with the SOLOv2 feature-branch tail fused
    (d2mi_group_norm_nhwc): up2 writes the nearest x2 upsample; accumulate_into
    adds the result into that tensor (returned).  Inference only (no grad)."""
    x = _f32c(x)
    gamma, beta = _f32c(gamma), _f32c(beta)
    _C.require_device(x, gamma, beta)
    N, H, W, C = x.shape
    oshape = (N, 2 * H, 2 * W, C) if up2 else (N, H, W, C)
    if accumulate_into is not None:
        y = accumulate_into
        if tuple(y.shape) != oshape or not y.is_contiguous() or y.dtype != torch.float32:
            raise ValueError(f"accumulate_into must be a contiguous f32 {oshape} tensor")
    else:
        y = torch.empty(oshape, dtype=torch.float32, device=x.device)
    lib = _C.lib()
    wsb = lib.d2mi_group_norm_workspace_size(N, H, W, C, int(num_groups))
    ws = _C.workspace(wsb, x.device)
    rc = lib.d2mi_group_norm_nhwc(_C.ptr(x), N, H, W, C, int(num_groups), _C.ptr(gamma),
                                  _C.ptr(beta), float(eps), int(bool(relu)), int(bool(up2)),
                                  int(accumulate_into is not None), _C.ptr(y), _C.ptr(ws), wsb,
                                  _C.stream_of(x.device))
    _C.check(rc, "d2mi_group_norm_nhwc")
    return y


def group_norm_levels(xs, num_groups, gamma, beta, eps, relu=False):
    """The same GroupNorm (+ ReLU) over up to 6 feature levels in one set of
    launches (d2mi_group_norm_nhwc_levels): per level ops.group_norm's
    arithmetic.  Inference only (no grad)."""
    xs = [_f32c(x) for x in xs]
    gamma, beta = _f32c(gamma), _f32c(beta)
    _C.require_device(gamma, beta, *xs)
    if not 1 <= len(xs) <= 6:
        raise ValueError(f"group_norm_levels takes 1..6 levels, got {len(xs)}")
    C = xs[0].shape[-1]
    dims, ys = [], []
    for x in xs:
        if x.dim() != 4 or x.shape[-1] != C:
            raise ValueError(f"every level must be [N, H, W, {C}], got {tuple(x.shape)}")
        dims += [x.shape[0], x.shape[1], x.shape[2]]
        ys.append(torch.empty_like(x))
    dm = _C.host_array(_C.ctypes.c_int32, dims)
    lib = _C.lib()
    wsb = lib.d2mi_group_norm_levels_workspace_size(dm, len(xs), C, int(num_groups))
    ws = _C.scratch(wsb, xs[0].device) if wsb else None
    xp = _C.host_array(_C.c_void_p, [x.data_ptr() for x in xs])
    yp = _C.host_array(_C.c_void_p, [y.data_ptr() for y in ys])
    rc = lib.d2mi_group_norm_nhwc_levels(xp, dm, len(xs), C, int(num_groups), _C.ptr(gamma),
                                         _C.ptr(beta), float(eps), int(bool(relu)), yp,
                                         _C.ptr(ws), wsb, _C.stream_of(xs[0].device))
    _C.check(rc, "d2mi_group_norm_nhwc_levels")
    return ys


# ------------------------------------------------------------ resize / SOLOv2
class _ResizeBilinearFn(torch.autograd.Function):
    """The half-pixel ResizeBilinear with a gradient (SOLOv2 training: the
    head's grid resamples of the FPN maps): forward on the HIP kernel, the
    adjoint of the same bilinear weights (half-pixel centres, edge-clamped;
    PyTorch's align_corners=False sampling is that rule) for the backward."""

    @staticmethod
    def forward(ctx, x, oh, ow):
        ctx.in_shape = tuple(x.shape)
        return resize_bilinear(x.detach(), (oh, ow))

    @staticmethod
    def backward(ctx, g):
        N, H, W, C = ctx.in_shape
        gi = torch.ops.aten.upsample_bilinear2d_backward(
            g.permute(0, 3, 1, 2).contiguous(), [g.shape[1], g.shape[2]], [N, C, H, W], False,
            None, None)
        return gi.permute(0, 2, 3, 1), None, None


def resize_bilinear_grad(x, size):
    """resize_bilinear (half-pixel) that autograd can differentiate."""
    if torch.is_grad_enabled() and x.requires_grad:
        return _ResizeBilinearFn.apply(x, int(size[0]), int(size[1]))
    return resize_bilinear(x, size)


def resize_bilinear(x, size, align_corners=False, half_pixel_centers=True):
    """TF ResizeBilinear on NHWC f32 (d2mi_resize_bilinear): x [N,H,W,C] ->
    [N, size[0], size[1], C]."""
    x = _f32c(x)
    _C.require_device(x)
    N, H, W, C = x.shape
    OH, OW = int(size[0]), int(size[1])
    y = torch.empty((N, OH, OW, C), dtype=torch.float32, device=x.device)
    rc = _C.lib().d2mi_resize_bilinear(_C.ptr(x), N, H, W, C, OH, OW, int(bool(align_corners)),
                                       int(bool(half_pixel_centers)), _C.ptr(y),
                                       _C.stream_of(x.device))
    _C.check(rc, "d2mi_resize_bilinear")
    return y


def solo_inference(cate_logits, kernels, mask_features, strides, out_hw, score_thresh=0.1,
                   mask_thresh=0.5, update_thresh=0.05, pre_nms_topk=500, max_detections=100,
                   nms_kernel="gaussian", nms_sigma=2.0, debug=None):
    """MaskKernelBranch.inference (solo_v2.py:476-627) on the HIP stages of
    csrc/solo.hip.  cate_logits[l] [N,S_l,S_l,K] (pre-sigmoid), kernels[l]
    [N,S_l,S_l,D], mask_features [N,Hm,Wm,D], strides[l] (the per-level
    sum_masks floor), out_hw the padded image size.  Returns masks uint8
    [N,max_det,OH,OW], boxes [N,max_det,4], scores, classes int64, is_valid.
    One host read (the live-cell counts that size the dynamic-conv GEMMs).
    debug: a dict to receive the intermediates (tests)."""
    if nms_kernel not in ("gaussian", "linear"):
        raise NotImplementedError(f"NMS kernel {nms_kernel} not implemented yet.")
    cate = [_f32c(t) for t in cate_logits]
    kern = [_f32c(t) for t in kernels]
    feats = _f32c(mask_features)
    _C.require_device(feats, *cate, *kern)
    N, K = cate[0].shape[0], cate[0].shape[-1]
    D = kern[0].shape[-1]
    _, Hm, Wm, D2 = feats.shape
    if D != D2:
        raise ValueError(f"kernel dims {D} != mask feature dims {D2}")
    P = Hm * Wm
    L = len(cate)
    grids = [int(t.shape[1]) for t in cate]
    T = sum(g * g for g in grids)
    dev = feats.device
    st = _C.stream_of(dev)
    lib = _C.lib()
    g_arr = _C.host_array(_C.ctypes.c_int32, grids)
    s_arr = _C.host_array(_C.c_float, [float(s) for s in strides])
    probs = torch.empty((N, T, K), dtype=torch.float32, device=dev)
    live_cells = torch.empty((N, T), dtype=torch.int32, device=dev)
    live_row = torch.empty((N, T), dtype=torch.int32, device=dev)
    live_count = torch.empty((N,), dtype=torch.int32, device=dev)
    rc = lib.d2mi_solo_cells(_C.host_array(_C.c_void_p, [t.data_ptr() for t in cate]), g_arr, L,
                             N, K, float(score_thresh), _C.ptr(probs), _C.ptr(live_cells),
                             _C.ptr(live_row), _C.ptr(live_count), st)
    _C.check(rc, "d2mi_solo_cells")
    counts = host_sync.read_ints(live_count)  # the one host synchronisation
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    R = offs[-1]
    row_off = torch.tensor(offs[:-1], dtype=torch.int32, device=dev)
    kern_all = torch.cat([k.reshape(N, -1, D) for k in kern], 1)  # [N, T, D]
    logits = torch.empty((max(R, 1), P), dtype=torch.float32, device=dev)
    for n in range(N):
        c = counts[n]
        if c == 0:
            continue
        rows = kern_all[n].index_select(0, live_cells[n, :c].long()).reshape(1, 1, c, D)
        # dynamic 1x1 conv (solo_v2.py:509-511): one MFMA GEMM per image,
        # [c, D] x [P, D]^T -> [c, P] written straight into the shared buffer
        conv2d_nhwc(rows, feats[n].reshape(1, 1, P, D), out=logits[offs[n]:offs[n + 1]].view(
            1, 1, c, P))
    sum_masks = torch.empty((max(R, 1),), dtype=torch.float32, device=dev)
    sum_scores = torch.empty_like(sum_masks)
    ev = KernelTimer.start()
    rc = lib.d2mi_solo_mask_stats(_C.ptr(logits), R, P, float(mask_thresh), _C.ptr(sum_masks),
                                  _C.ptr(sum_scores), st)
    KernelTimer.stop(ev, "solo_mask_stats", 4 * R * P)  # the dynamic-conv logits read once
    _C.check(rc, "d2mi_solo_mask_stats")
    k = int(min(pre_nms_topk, T * K))
    top_scores = torch.empty((N, k), dtype=torch.float32, device=dev)
    top_classes = torch.empty((N, k), dtype=torch.int64, device=dev)
    top_sum = torch.empty((N, k), dtype=torch.float32, device=dev)
    top_count = torch.empty((N,), dtype=torch.int32, device=dev)
    W64 = (P + 63) // 64
    bits = torch.empty((N, k, W64), dtype=torch.int64, device=dev)
    wsb = lib.d2mi_solo_select_workspace_size(N, T, K, k)
    ws = _C.workspace(wsb, dev)
    rc = lib.d2mi_solo_select(_C.ptr(probs), _C.ptr(live_row), _C.ptr(row_off), _C.ptr(logits),
                              _C.ptr(sum_masks), _C.ptr(sum_scores), g_arr, s_arr, L, N, K, P,
                              float(score_thresh), float(mask_thresh), k, _C.ptr(top_scores),
                              _C.ptr(top_classes), _C.ptr(top_sum), _C.ptr(top_count),
                              _C.ptr(bits), _C.ptr(ws), wsb, st)
    _C.check(rc, "d2mi_solo_select")
    # Matrix NMS (solo_v2.py:541-545) over the padded top-k rows, all images
    decayed = torch.empty((N, k), dtype=torch.float32, device=dev)
    mwsb = lib.d2mi_solo_matrix_nms_workspace_size(N, k)
    mws = _C.workspace(mwsb, dev)
    ev = KernelTimer.start()
    rc = lib.d2mi_solo_matrix_nms(_C.ptr(bits), _C.ptr(top_classes), _C.ptr(top_scores),
                                  _C.ptr(top_sum), N, k, P, 0 if nms_kernel == "gaussian" else 1,
                                  float(nms_sigma), _C.ptr(decayed), _C.ptr(mws), mwsb, st)
    if get_tuning("solo_mfma"):
        # the int8 MFMA intersections (r6): SURVEY 8d D4's 2 N^2 HW ops per
        # image (the reference's full M M^T; the kernel forms the upper
        # triangle) against the I8 MFMA peak
        KernelTimer.stop(ev, "solo_matrix_nms", 2 * N * k * k * P)
    else:
        # the AND + popcount tiles: the bit-packed masks read once (bytes)
        KernelTimer.stop(ev, "solo_matrix_nms_popcount", N * k * W64 * 8)
    _C.check(rc, "d2mi_solo_matrix_nms")
    OH, OW = int(out_hw[0]), int(out_hw[1])
    out_masks = torch.empty((N, max_detections, OH, OW), dtype=torch.uint8, device=dev)
    out_boxes = torch.empty((N, max_detections, 4), dtype=torch.float32, device=dev)
    out_scores = torch.empty((N, max_detections), dtype=torch.float32, device=dev)
    out_classes = torch.empty((N, max_detections), dtype=torch.int64, device=dev)
    out_valid = torch.empty((N, max_detections), dtype=torch.uint8, device=dev)
    fwsb = lib.d2mi_solo_finalize_workspace_size(N, max_detections, OH)
    fws = _C.workspace(fwsb, dev)
    ev = KernelTimer.start()
    rc = lib.d2mi_solo_finalize(_C.ptr(decayed), _C.ptr(top_classes), _C.ptr(top_count),
                                _C.ptr(bits), N, k, Hm, Wm, float(update_thresh),
                                int(max_detections), float(mask_thresh), OH, OW,
                                _C.ptr(out_masks), _C.ptr(out_boxes), _C.ptr(out_scores),
                                _C.ptr(out_classes), _C.ptr(out_valid), _C.ptr(fws), fwsb, st)
    # algorithmic bytes: the uint8 canvas written once (the bit masks are L2-resident)
    KernelTimer.stop(ev, "solo_paste", N * max_detections * OH * OW)
    _C.check(rc, "d2mi_solo_finalize")
    if debug is not None:
        debug.update(probs=probs, live_cells=live_cells, live_row=live_row, counts=counts,
                     row_off=offs, logits=logits[:R], sum_masks=sum_masks[:R],
                     sum_scores=sum_scores[:R], top_scores=top_scores, top_classes=top_classes,
                     top_sum=top_sum, top_count=top_count, mask_bits=bits, decayed=decayed)
    return out_masks, out_boxes, out_scores, out_classes, out_valid.bool()


# ------------------------------------------------------- fused post-processing
# host copies of the cell anchors (constant buffers, often on the GPU: one
# read per element was ~60 device-to-host syncs per training step)
_CELLS = {}


def _cell_values(c):
    """The float32 values of one level's cell anchors as a tuple.  A tensor
    keeps its host copy as an attribute of the tensor object itself (checked
    against its in-place version counter), so the copy lives and dies with
    that tensor: no cache key that another tensor at a reused address could
    match."""
    if not torch.is_tensor(c):
        return tuple(np.asarray(c, np.float32).reshape(-1).tolist())
    got = getattr(c, "_d2mi_host_cells", None)
    if got is None or got[0] != c._version:
        got = (c._version, tuple(c.detach().to(torch.float32).reshape(-1).cpu().tolist()))
        c._d2mi_host_cells = got
    return got[1]


def _cell_host_array(cell_anchors):
    """ctypes array of every level's cell anchors, cached by VALUE (tens of
    floats per level)."""
    key = tuple(_cell_values(c) for c in cell_anchors)
    got = _CELLS.get(key)
    if got is None:
        cells = [v for lv in key for v in lv]
        got = (_C.host_array(_C.c_float, cells), len(cells))
        if len(_CELLS) > 64:
            _CELLS.clear()
        _CELLS[key] = got
    return got


def _level_arrays(tensors, hw, strides, cell_anchors):
    L = len(tensors)
    ptrs = _C.host_array(_C.c_void_p, [t.data_ptr() for t in tensors])
    lhw = _C.host_array(_C.ctypes.c_int32, [v for h, w in hw for v in (int(h), int(w))])
    st = _C.host_array(_C.c_float, [float(s) for s in strides])
    cells, n = _cell_host_array(cell_anchors)
    return ptrs, lhw, st, cells, n // (4 * L)


def _image_strided(t):
    """t [N, H, W, C] f32 on the device, dense within each image (any image
    stride, e.g. a level view of a concatenated [N, sum HWC] buffer)."""
    N, H, W, C = t.shape
    return (t.dtype == torch.float32 and t.stride(3) == 1 and t.stride(2) == C
            and t.stride(1) == W * C and t.stride(0) >= H * W * C)


def rpn_proposals(logits, deltas, strides, cell_anchors, image_hw, pre_nms_topk, post_nms_topk,
                  nms_thresh, min_box_side_len=0.0, weights=(1.0, 1.0, 1.0, 1.0),
                  scale_clamp=_DEFAULT_SCALE_CLAMP):
    """find_top_rpn_proposals (rpn_outputs.py:29-132) fused with anchor
    generation and decode.  logits[l] [N,H,W,A], deltas[l] [N,H,W,A*4]; each
    dense within an image, any image stride (level views of the training
    head's concatenated outputs go in without copies: d2mi_rpn_proposals_ex)."""
    strided = (all(_image_strided(t) for t in list(logits) + list(deltas))
               and all(t.data_ptr() % 16 == 0 for t in deltas))
    if not strided:
        logits = [_f32c(t) for t in logits]
        deltas = [_f32c(t) for t in deltas]
    image_hw = _i32c(image_hw)
    _C.require_device(image_hw, *logits, *deltas)
    N = logits[0].shape[0]
    L = len(logits)
    hw = [(t.shape[1], t.shape[2]) for t in logits]
    lp, lhw, st, cells, A = _level_arrays(logits, hw, strides, cell_anchors)
    dp = _C.host_array(_C.c_void_p, [t.data_ptr() for t in deltas])
    dev = logits[0].device
    ob = torch.empty((N, post_nms_topk, 4), dtype=torch.float32, device=dev)
    os_ = torch.empty((N, post_nms_topk), dtype=torch.float32, device=dev)
    ov = torch.empty((N, post_nms_topk), dtype=torch.uint8, device=dev)
    wsb = _C.lib().d2mi_rpn_proposals_workspace_size(N, L, lhw, A, pre_nms_topk, post_nms_topk)
    ws = _C.workspace(wsb, dev)
    sl = _C.host_array(_C.ctypes.c_int64, [t.stride(0) for t in logits])
    sd = _C.host_array(_C.ctypes.c_int64, [t.stride(0) for t in deltas])
    rc = _C.lib().d2mi_rpn_proposals_ex(lp, dp, sl, sd, lhw, st, cells, L, A, N, _C.ptr(image_hw),
                                     int(pre_nms_topk), int(post_nms_topk), float(nms_thresh),
                                     float(min_box_side_len),
                                     _C.host_array(_C.c_float, [float(w) for w in weights]),
                                     float(scale_clamp), _C.ptr(ob), _C.ptr(os_), _C.ptr(ov),
                                     _C.ptr(ws), wsb, _C.stream_of(dev))
    _C.check(rc, "d2mi_rpn_proposals")
    return ob, os_, ov.bool()


def rpn_head_gather(ys, A):
    """d2mi_rpn_head_gather: the fused head's per-level outputs ys[l] [N, H, W, C]
    -> (logits [N, T*A], deltas [N, T*A, 4]) in the RPNOutputs layout."""
    ys = [_f32c(y) for y in ys]
    _C.require_device(*ys)
    N, C = ys[0].shape[0], ys[0].shape[-1]
    hw = [y.shape[1] * y.shape[2] for y in ys]
    T = sum(hw)
    dev = ys[0].device
    pl = torch.empty((N, T * A), dtype=torch.float32, device=dev)
    pd = torch.empty((N, T * A, 4), dtype=torch.float32, device=dev)
    rc = _C.lib().d2mi_rpn_head_gather(_C.host_array(_C.c_void_p, [y.data_ptr() for y in ys]),
                                       _C.host_array(_C.ctypes.c_int32, hw), len(ys), N, A, C,
                                       _C.ptr(pl), _C.ptr(pd), _C.stream_of(dev))
    _C.check(rc, "d2mi_rpn_head_gather")
    return pl, pd


def rpn_head_scatter(g_logits, g_deltas, shapes, A):
    """Adjoint of rpn_head_gather: -> per-level [N, H, W, C] gradients (every
    element written; either input may be None = zero)."""
    g_logits = _f32c(g_logits) if g_logits is not None else None
    g_deltas = _f32c(g_deltas) if g_deltas is not None else None
    ref = g_logits if g_logits is not None else g_deltas
    dev = ref.device
    N, C = shapes[0][0], shapes[0][-1]
    outs = [torch.empty(tuple(s), dtype=torch.float32, device=dev) for s in shapes]
    hw = [s[1] * s[2] for s in shapes]
    rc = _C.lib().d2mi_rpn_head_scatter(_C.ptr(g_logits), _C.ptr(g_deltas),
                                        _C.host_array(_C.ctypes.c_int32, hw), len(shapes), N, A, C,
                                        _C.host_array(_C.c_void_p, [o.data_ptr() for o in outs]),
                                        _C.stream_of(dev))
    _C.check(rc, "d2mi_rpn_head_scatter")
    return outs


def fast_rcnn_inference(logits, deltas, proposals, roi_img, roi_slot, num_images, P, image_hw,
                        weights, score_thresh, nms_thresh, topk_per_image,
                        cls_agnostic=False, scale_clamp=_DEFAULT_SCALE_CLAMP, nms_cls_agnostic=False):
    """FastRCNNOutputs.inference + fast_rcnn_inference (fast_rcnn.py:28-187,
    :359-395): softmax, decode, clip, threshold, class-offset NMS (plain NMS
    with nms_cls_agnostic, fast_rcnn.py:138-139), pad.  cls_agnostic: one
    class-agnostic box per ROI (deltas [R, 4])."""
    logits, deltas, proposals = _f32c(logits), _f32c(deltas), _f32c(proposals)
    roi_img, roi_slot, image_hw = _i32c(roi_img), _i32c(roi_slot), _i32c(image_hw)
    _C.require_device(logits, deltas, proposals, roi_img, roi_slot, image_hw)
    R, K1 = logits.shape
    K = K1 - 1
    N = int(num_images)
    dev = logits.device
    ob = torch.empty((N, topk_per_image, 4), dtype=torch.float32, device=dev)
    os_ = torch.empty((N, topk_per_image), dtype=torch.float32, device=dev)
    oc = torch.empty((N, topk_per_image), dtype=torch.int64, device=dev)
    ov = torch.empty((N, topk_per_image), dtype=torch.uint8, device=dev)
    oroi = torch.empty((N, topk_per_image), dtype=torch.int32, device=dev)
    wsb = _C.lib().d2mi_fast_rcnn_workspace_size(N, int(P), K, float(score_thresh),
                                                 int(topk_per_image))
    ws = _C.workspace(wsb, dev)
    rc = _C.lib().d2mi_fast_rcnn_inference(
        _C.ptr(logits), _C.ptr(deltas), _C.ptr(proposals), _C.ptr(roi_img), _C.ptr(roi_slot), R,
        N, int(P), K, int(bool(cls_agnostic)) | (int(bool(nms_cls_agnostic)) << 1), _C.ptr(image_hw),
        _C.host_array(_C.c_float, [float(w) for w in weights]), float(scale_clamp),
        float(score_thresh), float(nms_thresh), int(topk_per_image), _C.ptr(ob), _C.ptr(os_),
        _C.ptr(oc), _C.ptr(ov), _C.ptr(oroi), _C.ptr(ws), wsb, _C.stream_of(dev))
    _C.check(rc, "d2mi_fast_rcnn_inference")
    return ob, os_, oc, ov.bool(), oroi


def retinanet_inference(box_cls, box_delta, strides, cell_anchors, num_classes, topk_candidates,
                        score_threshold, nms_threshold, max_detections,
                        weights=(1.0, 1.0, 1.0, 1.0), scale_clamp=_DEFAULT_SCALE_CLAMP):
    """RetinaNetHead.inference (retinanet.py:285-387).  box_cls[l] [N,H,W,A*K],
    box_delta[l] [N,H,W,A*4]."""
    box_cls = [_f32c(t) for t in box_cls]
    box_delta = [_f32c(t) for t in box_delta]
    _C.require_device(*box_cls, *box_delta)
    N = box_cls[0].shape[0]
    L = len(box_cls)
    hw = [(t.shape[1], t.shape[2]) for t in box_cls]
    cp, lhw, st, cells, A = _level_arrays(box_cls, hw, strides, cell_anchors)
    bp = _C.host_array(_C.c_void_p, [t.data_ptr() for t in box_delta])
    dev = box_cls[0].device
    ob = torch.empty((N, max_detections, 4), dtype=torch.float32, device=dev)
    os_ = torch.empty((N, max_detections), dtype=torch.float32, device=dev)
    oc = torch.empty((N, max_detections), dtype=torch.int32, device=dev)
    ov = torch.empty((N, max_detections), dtype=torch.uint8, device=dev)
    wsb = _C.lib().d2mi_retinanet_workspace_size(N, L, lhw, A, int(num_classes),
                                                 int(topk_candidates))
    ws = _C.workspace(wsb, dev)
    ev = KernelTimer.start()
    rc = _C.lib().d2mi_retinanet_inference(
        cp, bp, lhw, st, cells, L, A, int(num_classes), N, int(topk_candidates),
        float(score_threshold), float(nms_threshold), int(max_detections),
        _C.host_array(_C.c_float, [float(w) for w in weights]), float(scale_clamp), _C.ptr(ob),
        _C.ptr(os_), _C.ptr(oc), _C.ptr(ov), _C.ptr(ws), wsb, _C.stream_of(dev))
    # algorithmic bytes: the dense logit scan, 4 B per (anchor, class) score
    # (64.5 MB per image at 1333x800)
    KernelTimer.stop(ev, "retinanet_postprocess", 4 * sum(t.numel() for t in box_cls))
    _C.check(rc, "d2mi_retinanet_inference")
    return ob, os_, oc, ov.bool()


# ------------------------------------------------------------- mask pasting
def paste_masks(box_masks, boxes, out_shape, valid=None, yx_scale=None, threshold=0.5):
    """reframe_box_masks_to_image_masks (lib/structures/mask_ops.py:7-56) with
    the threshold of detector_postprocess (postprocessing.py:47-49) fused:
    box_masks [D, mh, mw] f32 probabilities, boxes [D, 4] yxyx absolute,
    out_shape (H, W) canvas; valid [D] bool (False rows -> zeros); yx_scale
    [D, 2] f32 per-box (sy, sx) applied first ("fixed" format).
    Returns [D, H, W] uint8."""
    box_masks = _f32c(box_masks)
    boxes = _f32c(boxes)
    tensors = [box_masks, boxes]
    if valid is not None:
        valid = valid.to(torch.uint8).contiguous()
        tensors.append(valid)
    if yx_scale is not None:
        yx_scale = _f32c(yx_scale)
        tensors.append(yx_scale)
    _C.require_device(*tensors)
    D, mh, mw = box_masks.shape
    H, W = int(out_shape[0]), int(out_shape[1])
    out = torch.empty((D, H, W), dtype=torch.uint8, device=boxes.device)
    ev = KernelTimer.start()
    rc = _C.lib().d2mi_paste_masks(_C.ptr(box_masks), _C.ptr(boxes), _C.ptr(yx_scale),
                                   _C.ptr(valid), D, mh, mw, H, W, float(threshold),
                                   _C.ptr(out), _C.stream_of(boxes.device))
    # algorithmic bytes: the u8 canvas written + the box masks read
    KernelTimer.stop(ev, "paste_masks", D * H * W + box_masks.numel() * 4)
    _C.check(rc, "d2mi_paste_masks")
    return out


def wgrad_skinny(x, g, with_bias=True, accumulate_into=None):
    """1x1-conv weight (+ bias) gradient for Cout <= 16 over all pixels:
    x [..., Cin], g [..., Cout] -> (gw [1, 1, Cin, Cout] HWIO, gb [Cout] or None).
    accumulate_into: a (gw, gb) pair of an earlier call to add this one into
    (old + new, in place; returned)."""
    x, g = _f32c(x), _f32c(g)
    _C.require_device(x, g)
    Cin, Cout = x.shape[-1], g.shape[-1]
    P = x.numel() // Cin
    if g.numel() != P * Cout:
        raise ValueError(f"wgrad_skinny: {tuple(x.shape)} vs {tuple(g.shape)}")
    if accumulate_into is not None:
        gw, gb = accumulate_into
        if (tuple(gw.shape) != (1, 1, Cin, Cout) or not gw.is_contiguous()
                or (gb is None) == with_bias):
            raise ValueError("wgrad_skinny: accumulate_into does not match this gradient")
    else:
        gw = torch.empty((1, 1, Cin, Cout), dtype=torch.float32, device=x.device)
        gb = torch.empty((Cout,), dtype=torch.float32, device=x.device) if with_bias else None
    wsb = _C.lib().d2mi_wgrad_skinny_workspace_size(P, Cin, Cout)
    ws = _C.workspace(wsb, x.device)
    ev = KernelTimer.start()
    rc = _C.lib().d2mi_wgrad_skinny_ex(_C.ptr(x), _C.ptr(g), P, Cin, Cout, _C.ptr(gw), _C.ptr(gb),
                                       int(accumulate_into is not None), _C.ptr(ws), wsb,
                                       _C.stream_of(x.device))
    # algorithmic bytes: x and g read once
    KernelTimer.stop(ev, "wgrad_skinny", 4 * P * (Cin + Cout))
    _C.check(rc, "d2mi_wgrad_skinny")
    return gw, gb


def wgrad_skinny_levels(xs, gs, with_bias=True):
    """wgrad_skinny of several calls sharing one weight, summed in list order
    (d2mi_wgrad_skinny_levels: one partial launch + one reduce; bit-identical
    to the calls one by one with accumulate_into after the first).  xs[l]
    [..., Cin] 16-B aligned with Cin % 4 == 0, gs[l] [..., Cout]."""
    xs = [_f32c(x) for x in xs]
    gs = [_f32c(g) for g in gs]
    _C.require_device(*xs, *gs)
    Cin, Cout = xs[0].shape[-1], gs[0].shape[-1]
    Ps = [x.numel() // Cin for x in xs]
    for x, g, P in zip(xs, gs, Ps):
        if x.shape[-1] != Cin or g.numel() != P * Cout:
            raise ValueError(f"wgrad_skinny_levels: {tuple(x.shape)} vs {tuple(g.shape)}")
    dev = xs[0].device
    gw = torch.empty((1, 1, Cin, Cout), dtype=torch.float32, device=dev)
    gb = torch.empty((Cout,), dtype=torch.float32, device=dev) if with_bias else None
    Pa = _C.host_array(_C.ctypes.c_int32, Ps)
    lib = _C.lib()
    wsb = lib.d2mi_wgrad_skinny_levels_workspace_size(Pa, len(xs), Cin, Cout)
    ws = _C.scratch(wsb, dev)
    ev = KernelTimer.start()
    rc = lib.d2mi_wgrad_skinny_levels(_C.host_array(_C.c_void_p, [x.data_ptr() for x in xs]),
                                      _C.host_array(_C.c_void_p, [g.data_ptr() for g in gs]), Pa,
                                      len(xs), Cin, Cout, _C.ptr(gw), _C.ptr(gb), 0, _C.ptr(ws),
                                      wsb, _C.stream_of(dev))
    KernelTimer.stop(ev, "wgrad_skinny", 4 * sum(Ps) * (Cin + Cout))
    _C.check(rc, "d2mi_wgrad_skinny_levels")
    return gw, gb


def skinny_levels_ok(x):
    """Whether a level's input can join wgrad_skinny_levels."""
    return x.dtype == torch.float32 and x.is_contiguous() and x.shape[-1] % 4 == 0 \
        and x.data_ptr() % 16 == 0


def column_sum(x):
    """Sum over every leading dim of x [..., C] -> [C] (fixed order)."""
    x = _f32c(x)
    _C.require_device(x)
    C = x.shape[-1]
    rows = x.numel() // C
    out = torch.empty((C,), dtype=torch.float32, device=x.device)
    wsb = _C.lib().d2mi_column_sum_workspace_size(rows, C)
    ws = _C.workspace(wsb, x.device)
    rc = _C.lib().d2mi_column_sum(_C.ptr(x), rows, C, _C.ptr(out), _C.ptr(ws), wsb,
                                  _C.stream_of(x.device))
    _C.check(rc, "d2mi_column_sum")
    return out
