"""Conv2D / ConvTranspose2D with the reference's constructor surface
(lib/layers/convolutional.py:119-263, :747-893).

Activations are NHWC, weights are HWIO ``[k, k, in/groups, out]`` (the
reference variable layout; ConvTranspose2D keeps TF's ``[k, k, out, in]``).
``impl="mfma"`` runs the forward pass on the hand-written gfx950 MFMA
implicit-GEMM kernel (d2mi_conv2d_nhwc) — the FPN lateral/output convs, the
RPN head and the mask head use it — and raises if the tensor is not on the GPU.
``impl="torch"`` is stock PyTorch-ROCm conv2d in channels_last, used for the
backbone (a caller of the hot path, outside its scope).
``impl="auto"`` picks mfma when the shape is eligible (no groups/dilation,
Cin % 4 == 0) and the input is on the GPU; ``impl="mfma"`` with Cin % 4 != 0
runs with zero channels appended.
Backward of the mfma path: dgrad on the same MFMA kernel (flipped kernel);
wgrad on the MFMA wgrad kernel or hipBLASLt / MIOpen, whichever measured
faster for the shape (see _wgrad); stride-2 KxK dgrad and Cout % 4 != 0 use
torch.nn.grad.
"""
import os

import torch
import torch.nn.functional as F

from ..utils.arg_scope import add_arg_scope
from . import handoff
from . import initializers as init
from . import ops
from .activation import get_activation, is_relu
from .base import Layer
from .normalization import BatchNorm


def fix_padding(inputs, kernel_size, padding="SAME", rate=1):
    """Explicit symmetric 'SAME' padding (convolutional.py:12-23): NHWC zero pad."""
    if padding == "SAME" and kernel_size != 1:
        pb, pe = same_pads(kernel_size, rate)
        inputs = F.pad(inputs, (0, 0, pb, pe, pb, pe))
    return inputs


def same_pads(kernel_size, rate=1):
    k_eff = kernel_size + (kernel_size - 1) * (rate - 1)
    pad_total = k_eff - 1
    pb = pad_total // 2
    return pb, pad_total - pb


def _dgrad(gy, w, x_shape, stride, pb, pe, relu_gate=None, add=None, add2=None):
    """Input gradient (+ add, then the relu_gate mask, when given).  Stride 1:
    a forward conv of gy with the spatially flipped kernel — whose HWIO layout IS the packed [KH, KW, out', in'] layout
    of the transposed conv, flipped by the kernel's tap indexing (kFlipTaps) —
    on the MFMA kernel, padded (KH-1-pb, KH-1-pe).
    1x1 stride s: the MFMA GEMM gy . W^T on the strided grid, scattered into
    zeros.  Anything else: torch.nn.grad (MIOpen)."""
    KH, KW, Cin, Cout = w.shape
    gy = gy.contiguous()
    if add2 is not None:  # (dgrad + add) + add2, gated: the strided 1x1 scatter only
        if not (KH == 1 and KW == 1 and pb == 0 and pe == 0 and stride > 1 and Cin % 4 == 0
                and Cout % 4 == 0):
            gx = _dgrad(gy, w, x_shape, stride, pb, pe, add=add).add_(add2)
            return gx if relu_gate is None else torch.ops.aten.threshold_backward(gx, relu_gate, 0.0)
        g = ops.conv2d_nhwc(gy, w.detach().contiguous(), None, 1, (0, 0))
        return ops.stride_scatter(g, x_shape, stride, add, add2, relu_gate)
    if KH == KW and Cout % 4 == 0:
        if stride == 1 and max(pb, pe) <= KH - 1:
            # the flip is an index flip inside the kernel (no flipped copy)
            return ops.conv2d_nhwc(gy, w.detach().contiguous(), None, 1,
                                   (KH - 1 - pb, KH - 1 - pe), flip_taps=KH > 1,
                                   residual=add, relu_gate=relu_gate)
        if KH == 1 and pb == 0 and pe == 0:
            g = ops.conv2d_nhwc(gy, w.detach().contiguous(), None, 1, (0, 0))
            if Cin % 4 == 0:  # zero holes + scatter (+ add) (+ gate) in one pass
                return ops.stride_scatter(g, x_shape, stride, add, gate=relu_gate)
            gx = torch.zeros(x_shape, dtype=gy.dtype, device=gy.device)
            gx[:, ::stride, ::stride] = g
            gx = gx if add is None else gx.add_(add)
            return gx if relu_gate is None else torch.ops.aten.threshold_backward(gx, relu_gate, 0.0)
    if relu_gate is not None:
        raise ValueError("relu_gate is fused into the stride-1 MFMA dgrad / the 1x1 scatter only")
    xin_shape = (x_shape[0], x_shape[3], x_shape[1] + pb + pe, x_shape[2] + pb + pe)
    gx = torch.nn.grad.conv2d_input(xin_shape, w.permute(3, 2, 0, 1), gy.permute(0, 3, 1, 2),
                                    stride, 0)
    gx = gx[:, :, pb:gx.shape[2] - pe, pb:gx.shape[3] - pe].permute(0, 2, 3, 1)
    return gx if add is None else gx + add


_WGRAD_1X1_MIN_P = int(os.environ.get("D2MI_WGRAD_1X1_MIN_P", "8192"))


def _wgrad(x, gy, w_shape, stride, pb, pe, want_bias=False, accumulate_into=None):
    """(weight gradient HWIO, bias gradient or None).

    accumulate_into: (gw, gb) of earlier calls of the same shared weight
    (gb None without a bias): this call's gradient is added into them --
    inside the MFMA wgrad's reduce pass where it runs, else by an in-place
    add -- and the accumulators are returned (gb None when this path made
    no bias gradient: the caller adds its column sum).

    Routed by measurement (tools/bench_kernels.py --only wgrad, MI355X):
    with split products (the default, ops.CONV_MATH) every KxK and every 1x1
    over >= 8k output pixels runs on the MFMA wgrad kernel (bias gradient
    fused; FPN p2 3x3 154 TF/s vs MIOpen's 122, mask-head 3x3 147 vs 110);
    smaller 1x1 -> X^T . dY as one hipBLASLt GEMM.  With f32 products the
    KxK go to MIOpen's igemm wrw, which beats the f32 MFMA kernel there."""
    KH, KW, Cin, Cout = w_shape
    split = ops.CONV_MATH == "split"
    eligible = Cin % 4 == 0 and Cout % 4 == 0
    acc_w, acc_b = accumulate_into if accumulate_into is not None else (None, None)

    def mfma(k, pads):
        if want_bias and (acc_w is None or acc_b is not None):
            acc = (acc_w, acc_b) if acc_w is not None else None
            return ops.conv2d_wgrad(x, gy, k, stride, pads, with_bias=True, accumulate_into=acc)
        return ops.conv2d_wgrad(x, gy, k, stride, pads, accumulate_into=acc_w), None

    def added(gw):  # a path without the fused accumulate
        return (gw if acc_w is None else acc_w.add_(gw)), None

    if KH == 1 and KW == 1 and pb == 0 and pe == 0:
        P = gy.numel() // Cout
        # tools/exp_wgrad_1x1.py: MFMA from 8400 pixels (res4: 54 vs 64-79 us
        # on hipBLASLt), and the strided 1024->2048 at 2100; hipBLASLt below
        if eligible and (P >= _WGRAD_1X1_MIN_P or (stride > 1 and Cin * Cout >= 2 ** 21)):
            return mfma(1, (0, 0))
        xs = x if stride == 1 else x[:, ::stride, ::stride]
        xs = xs.reshape(-1, Cin)
        return added(torch.mm(xs.t(), gy.reshape(-1, Cout)).reshape(1, 1, Cin, Cout))
    if split and eligible and KH == KW and 6 * max(x.numel(), gy.numel()) < 2 ** 31:
        return mfma(KH, (pb, pe))
    xin = F.pad(x, (0, 0, pb, pe, pb, pe)) if (pb or pe) else x
    gw = torch.nn.grad.conv2d_weight(xin.permute(0, 3, 1, 2), (Cout, Cin, KH, KW),
                                     gy.permute(0, 3, 1, 2), stride, 0)
    return added(gw.permute(2, 3, 1, 0))


def _wgrad_shared(acc, x, gy, w_shape, stride, pb, pe, want_bias):
    """One call's share of a weight used by several calls of one forward
    (``wacc`` = {"n": calls, "k": done}: the RPN head's 3x3 over the FPN
    levels): its (gw, gb) go into the accumulator (the reduce pass adds them:
    old + new, autograd's order for the summed gradients); every call but the
    last returns (None, None), the last the sums."""
    acc["k"] += 1
    if acc["k"] == 1:
        # every call's backward must run in this pass, else the gradient
        # never leaves and a stale buffer would poison a later backward
        handoff.expect_complete(acc, lambda a: a["k"] == 0,
                                lambda a: (a.pop("buf", None), a.__setitem__("k", 0)),
                                "shared conv weight-gradient calls")
    buf = acc.get("buf")
    gw, gb = _wgrad(x, gy, w_shape, stride, pb, pe, want_bias, accumulate_into=buf)
    if want_bias and gb is None:
        cs = ops.column_sum(gy)
        gb = cs if buf is None or buf[1] is None else buf[1].add_(cs)
    acc["buf"] = (gw, gb)
    if acc["k"] < acc["n"]:
        return None, None
    acc.pop("buf")
    acc["k"] = 0  # (a second backward of the same graph starts over)
    return gw, gb


# r6: {"stream": a side stream} while the graphed training step captures its
# backward (engine/graphed.py): every MFMA conv's weight gradient is issued
# there, beside its data gradient, so the replayed graph runs the two
# concurrently (a replayed graph runs forked branches in parallel,
# tools/graph_parallel_probe.py).  Empty in eager steps: a per-layer stream
# fork costs host time there (r2 measured +3.7 %), and a replay pays none.
WGRAD_STREAM = {}


def _wgrad_of(ctx, x, gy, w, stride, pb, pe, want_b):
    """(weight, bias) gradient of _ConvMFMAFn's backward, None where not needed."""
    gw = gb = None
    if ctx.needs_input_grad[1] and ctx.wacc is not None:
        gw, gb = _wgrad_shared(ctx.wacc, x, gy, w.shape, stride, pb, pe, want_b)
    else:
        if ctx.needs_input_grad[1]:
            gw, gb = _wgrad(x, gy, w.shape, stride, pb, pe, want_b)
        if want_b and gb is None:
            gb = ops.column_sum(gy)
    return gw, gb


def _gate_eligible(w_shape, stride, pb, pe):
    KH, KW, _, Cout = w_shape
    return KH == KW and Cout % 4 == 0 and stride == 1 and max(pb, pe) <= KH - 1


class _ConvMFMAFn(torch.autograd.Function):
    """Fused-ReLU chains: a conv with a fused ReLU tags its output.  A consumer
    conv called with gate_input=True (the caller's declaration that it is the
    SOLE consumer of that ReLU output: the bottleneck's conv2 / conv3, the mask
    head's conv chain and deconv) applies the producer's ReLU mask in its own
    dgrad epilogue (kMaskByResidual) and flags it; the producer then skips its
    threshold_backward.  Without the declaration nothing is fused.

    Residual-gradient hand-off (the bottleneck's identity shortcut): the conv
    that adds ``residual`` is given a dict ``res_grad_to`` and the conv that
    reads the same tensor as its input the same dict as ``grad_from``.  The
    adder's backward (always first: the reader's backward waits for the chain
    in between) leaves the residual's gradient there instead of returning
    it, and the reader adds it inside its dgrad epilogue -- before the ReLU
    gate, so  gx = (dgrad + g_res) * (x > 0)  is one pass and autograd never
    materialises the sum.

    Pair hand-off (``pair_grad``: the bottleneck's conv1 and projection
    shortcut, both reading x): whichever backward runs first leaves its input
    gradient in the shared dict and returns none for x; the second adds it in
    its own dgrad epilogue / stride scatter and returns the sum.  Both always
    run once the block output has a gradient (each feeds it)."""

    @staticmethod
    def forward(ctx, x, w_hwio, bias, w_packed, stride, pads, relu, topdown, residual=None,
                relu_after=False, gate_input=False, res_grad_to=None, grad_from=None,
                pair_grad=None, join=None, wacc=None):
        has_add = topdown is not None or residual is not None
        if relu and has_add and not relu_after:
            raise ValueError("relu(conv) + add is not differentiable here; use relu_after_add")
        y = ops.conv2d_nhwc(x, w_packed, bias, stride, pads, relu, topdown, residual,
                            relu_after_add=relu_after)
        ctx.save_for_backward(x, w_hwio, y if relu else None)
        ctx.conf = (stride, pads, relu, bias is not None, topdown is not None, residual is not None)
        ctx.in_info = getattr(x, "_d2mi_relu_info", None) if gate_input else None
        ctx.res_grad_to = res_grad_to if residual is not None else None
        ctx.grad_from = grad_from
        ctx.pair_grad = pair_grad
        # FPN top-down hand-off (modeling/necks/fpn.py TD_HANDOFF): the merged
        # map's output conv (pair_grad {"td": True}) and the finer lateral that
        # reads it as its top-down input -- both MFMA convs, registered here
        if pair_grad is not None and pair_grad.get("td"):
            pair_grad["mfma"] = True
        tdp = getattr(topdown, "_d2mi_td_pair", None) if topdown is not None else None
        ctx.td_pair = (tdp if tdp is not None and tdp.get("mfma") and topdown.requires_grad
                       else None)
        if ctx.td_pair is not None:
            ctx.td_pair["lat_mfma"] = True
        ctx.join = join
        ctx.wacc = wacc  # a weight shared by several calls: _wgrad_shared
        # the producer's ReLU tag, used if a join is registered by backward time
        ctx.relu_cand = getattr(x, "_d2mi_relu_info", None)
        ctx.out_info = None
        if relu:  # (forward runs with grad mode off: tag unconditionally)
            ctx.out_info = {"masked": False}
            y._d2mi_relu_info = ctx.out_info
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        stride, (pb, pe), relu, has_bias, has_td, has_res = ctx.conf
        if relu and not (ctx.out_info is not None and ctx.out_info["masked"]):
            # relu is the last op whenever an add is fused (relu_after)
            gy = torch.ops.aten.threshold_backward(gy, y, 0.0)
        gtd = None
        if has_td and gy.shape[-1] % 4 == 0:
            gtd = ops.upsample2x_grad(gy)
        elif has_td:
            N, OH, OW, C = gy.shape
            g = F.pad(gy, (0, 0, 0, OW % 2, 0, OH % 2))
            gtd = g.reshape(N, (OH + 1) // 2, 2, (OW + 1) // 2, 2, C).sum((2, 4))
        if gtd is not None and ctx.td_pair is not None and ctx.needs_input_grad[7]:
            # the merged map's other reader is its output conv: first of the
            # two leaves its gradient, the second adds it (the output conv in
            # its dgrad epilogue) -- autograd's sum of the two, no add launch
            other = ctx.td_pair.pop("g", None)
            if other is None:
                handoff.deposit(ctx.td_pair, "g", gtd, "FPN top-down")
                gtd = None
            else:
                gtd = gtd + other
        gres = gy if has_res and ctx.needs_input_grad[8] else None
        if gres is not None and ctx.res_grad_to is not None:
            handoff.deposit(ctx.res_grad_to, "g", gres, "residual")  # taken by the conv reading it
            gres = None
        gx = gw = gb = None
        want_b = has_bias and ctx.needs_input_grad[2]
        side = WGRAD_STREAM.get("stream")
        main = None
        if side is not None and ctx.needs_input_grad[1] and gy.is_cuda:
            # r6: the weight gradient on the side stream, issued BEFORE the
            # data gradient, so that the two run concurrently (the replayed
            # graph has both branches); joined at the end of this backward
            main = torch.cuda.current_stream(gy.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                gw, gb = _wgrad_of(ctx, x, gy, w, stride, pb, pe, want_b)
        if ctx.needs_input_grad[0] and _join_active(ctx):
            gx = _join_backward(ctx, gy, x, w, stride, pb, pe)
        elif ctx.needs_input_grad[0]:
            add = ctx.grad_from.pop("g", None) if ctx.grad_from is not None else None
            pair = ctx.pair_grad
            if pair is not None and pair.get("td") and not pair.get("lat_mfma"):
                pair = None  # (an FPN output conv whose map no MFMA lateral reads)
            deposit = False
            deferred = None
            gated = ctx.in_info is not None and _gate_eligible(w.shape, stride, pb, pe)
            if pair is not None:
                other = pair.pop("g", None)
                if isinstance(other, ops.DeferredPixels):
                    # the ROI poolers' pixel pass of this level, run into this
                    # dgrad's full map afterwards (no add here); a gated or
                    # already-adding dgrad takes the pooled map instead
                    if add is None and not gated:
                        deferred, other = other, None
                    else:
                        other = other.materialize()
                if other is None and deferred is None:
                    deposit = True  # first of the pair: no gate, no add
                elif other is None:
                    pass
                elif add is None:
                    add = other
                else:
                    add = add + other
            info = None if deposit else ctx.in_info
            if info is not None and _gate_eligible(w.shape, stride, pb, pe):
                gx = _dgrad(gy, w, x.shape, stride, pb, pe, relu_gate=x, add=add)
                info["masked"] = True
            else:
                gx = _dgrad(gy, w, x.shape, stride, pb, pe, add=add)
            if deferred is not None:
                gx = deferred.add_into(gx.contiguous())
            if deposit:
                handoff.deposit(pair, "g", gx, "pair")
                gx = None
        if main is not None:
            main.wait_stream(side)
            for t in (gw, gb):  # (made on the side stream, used on this one)
                if t is not None:
                    t.record_stream(main)
        else:
            gw, gb = _wgrad_of(ctx, x, gy, w, stride, pb, pe, want_b)
        return (gx, gw, gb, None, None, None, None, gtd, gres, None, None, None, None, None, None,
                None)


def _join_active(ctx):
    p = ctx.join if ctx.join is not None else ctx.pair_grad
    return p is not None and p.get("join", False) and ctx.grad_from is None


def _join_backward(ctx, gy, x, w, stride, pb, pe):
    """Input gradient of a conv in a three-consumer join: a ReLU output x (a
    ResNet stage output) read by the next stage's conv1 / projection-shortcut
    pair AND by the FPN lateral (``join``, registered by the FPN forward in
    the pair's dict).  Autograd would form  lat + (pair2 + pair1)  and then
    the producer's threshold_backward; here
      * the first pair member deposits its gradient ("g", as without a join);
      * the second pair member forms  s = dgrad + g ; if the lateral's
        gradient is already there it returns  gate((s) + lat)  (one scatter
        pass for a strided 1x1), else it deposits s ("sum");
      * the lateral returns  gate(dgrad + s)  if s is there, else it deposits
        its own dgrad ("lat").
    The last one applies the producer's ReLU mask in the same pass and flags
    it (the producer then skips its threshold_backward), so the sum and the
    gate are bit-identical to the autograd formulation.  Members that
    deposit return None for x."""
    info = ctx.relu_cand
    if ctx.join is not None:  # the lateral
        p = ctx.join
        s = p.pop("sum", None)
        if s is None:
            handoff.deposit(p, "lat", _dgrad(gy, w, x.shape, stride, pb, pe), "join (lateral)")
            return None
        p["last"] = "lateral"  # (tests: which member completed the join)
        if info is not None and _gate_eligible(w.shape, stride, pb, pe):
            gx = _dgrad(gy, w, x.shape, stride, pb, pe, relu_gate=x, add=s)
            info["masked"] = True
            return gx
        return _dgrad(gy, w, x.shape, stride, pb, pe, add=s)
    p = ctx.pair_grad
    other = p.pop("g", None)
    if isinstance(other, ops.DeferredPixels):
        other = other.materialize()
    if other is None:  # first of the pair
        handoff.deposit(p, "g", _dgrad(gy, w, x.shape, stride, pb, pe), "join (pair)")
        return None
    lat = p.pop("lat", None)
    if lat is None:
        handoff.deposit(p, "sum", _dgrad(gy, w, x.shape, stride, pb, pe, add=other), "join (sum)")
        return None
    p["last"] = "pair"
    gate = x if info is not None else None
    gx = _dgrad(gy, w, x.shape, stride, pb, pe, relu_gate=gate, add=other, add2=lat)
    if info is not None:
        info["masked"] = True
    return gx


class FoldGroup:
    """The trainable Conv2D + FrozenBN layers of one network folded together:
    the first of them to run in a training forward folds all of them with
    ops.fold_frozen_bn_many (one launch, and one backward pair once every
    gradient has arrived, instead of three launches per layer); each layer
    then takes its own result once.  A layer whose parameters changed since
    (new version) or whose result was already taken (a second forward) makes
    the next fetch refold the group."""
    ENABLED = True

    def __init__(self, layers):
        self.layers = list(layers)
        self.slots = {}
        for layer in self.layers:
            layer._fold_group = self

    @classmethod
    def attach(cls, module):
        layers = [m for m in module.modules()
                  if isinstance(m, Conv2D) and isinstance(m.normalizer_fn, BatchNorm)]
        return cls(layers) if layers else None

    def fetch(self, layer):
        s = self.slots.get(id(layer))
        if s is None or s[3] or s[4] != layer._param_key():
            self._fold()
            s = self.slots.get(id(layer))
            if s is None:
                return None
        out = (s[0], s[1], s[2])
        self.slots[id(layer)] = [None, None, None, True, s[4]]
        return out

    def _fold(self):
        members = [m for m in self.layers if m.weights.is_cuda and m.fold_trainable()]
        entries = []
        for m in members:
            n = m.normalizer_fn
            entries.append((m.weights, m.bias, n.gamma, n.beta, n.moving_mean, n.moving_variance,
                            n.epsilon, m.wants_packed()))
        outs = ops.fold_frozen_bn_many(entries)
        self.slots = {id(m): [w, b, p, False, m._param_key()] for m, (w, b, p) in zip(members, outs)}


class PackGroup:
    """The un-normalised MFMA convs of one model (FPN, RPN head, ROI heads):
    their packed weight copies are refreshed together.  A layer joins on its
    first packed_weights() call; the first fetch that finds its layer's
    parameters changed (the optimizer stepped) repacks EVERY member whose
    parameters changed in one launch (ops.pack_conv_weights_many) instead of
    one launch per layer."""
    ENABLED = True

    def __init__(self):
        self.members = []

    @classmethod
    def attach(cls, module):
        layers = [m for m in module.modules()
                  if isinstance(m, Conv2D) and not isinstance(m.normalizer_fn, BatchNorm)]
        if not layers:
            return None
        g = cls()
        for m in layers:
            m._pack_group = g
        return g

    def fetch(self, layer):
        if not any(m is layer for m in self.members):
            self.members.append(layer)
        key = layer._pack_key(layer.weights)
        if layer._packed is not None and layer._packed_key == key:
            return layer._packed
        stale, keys = [], []
        for m in self.members:
            k = key if m is layer else m._pack_key(m.weights)
            if m._packed is None or m._packed_key != k:
                stale.append(m)
                keys.append(k)
        outs = ops.pack_conv_weights_many([m.weights.detach() for m in stale])
        for m, k, o in zip(stale, keys, outs):
            m._packed, m._packed_key = o, k
        return layer._packed


@add_arg_scope
class Conv2D(Layer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding="SAME", rate=1,
                 num_groups=1, use_bias=True, activation=None, normalizer=None,
                 normalizer_params=None, weights_initializer=None, weights_regularizer=None,
                 bias_initializer=None, bias_regularizer=None, variables_collections=None,
                 trainable=True, outputs_collections=None, impl="mfma", **kwargs):
        padding = padding.upper()
        if padding not in ("SAME", "VALID"):
            raise ValueError('"padding" must be "SAME" or "VALID."')
        if in_channels % num_groups != 0:
            raise ValueError(f'"in_channels" {in_channels} is not divisible by "num_groups" {num_groups}.')
        if out_channels % num_groups != 0:
            raise ValueError(f'"out_channels" {out_channels} is not divisible by "num_groups" {num_groups}.')
        super().__init__(in_channels=in_channels, out_channels=out_channels,
                         kernel_size=kernel_size, stride=stride, padding=padding, rate=rate,
                         num_groups=num_groups, use_bias=use_bias, activation=activation,
                         normalizer=normalizer, normalizer_params=normalizer_params,
                         weights_initializer=weights_initializer,
                         weights_regularizer=weights_regularizer,
                         bias_initializer=bias_initializer, bias_regularizer=bias_regularizer,
                         trainable=trainable, impl=impl, **kwargs)
        self.build()

    def build(self):
        shape = (self.kernel_size, self.kernel_size, self.in_channels // self.num_groups,
                 self.out_channels)
        w = torch.empty(shape, dtype=torch.float32)
        (self.weights_initializer or init.variance_scaling(2.0, distribution="untruncated_normal"))(w)
        self.weights = torch.nn.Parameter(w, requires_grad=self.trainable)
        if self.use_bias:
            b = torch.zeros(self.out_channels)
            if self.bias_initializer is not None:
                self.bias_initializer(b)
            self.bias = torch.nn.Parameter(b, requires_grad=self.trainable)
        else:
            self.bias = None
        self.normalizer_fn = None
        if self.normalizer is not None:
            p = dict(self.normalizer_params or {})
            p["channels"] = self.out_channels
            self.normalizer_fn = self.normalizer(**p)
        self.act_fn = get_activation(self.activation)
        self._packed = None
        self._packed_key = None

    def _mfma_eligible(self, x, padded=False):
        # impl="mfma" with Cin % 4 != 0 (e.g. SOLOv2's 256 + 2 coordinate
        # channels) runs with zero channels appended to the input and the
        # weights (exact: the extra products are 0); "auto" keeps such convs
        # (the 3-channel stem) on MIOpen
        return (x.is_cuda and self.num_groups == 1 and self.rate == 1
                and (padded or self.in_channels % 4 == 0))

    def _key_tensors(self):
        """(weights, the other tensors the fold reads), looked up once (the
        module attribute lookups are host time on every conv call)."""
        kt = self.__dict__.get("_key_ts")
        w = self.weights
        # (re-looked up when the weights move: .to() / .cuda() also replace
        # the normalizer's buffers)
        if kt is None or kt[0] is not w or kt[2] != w.data_ptr():
            rest = [self.bias] if self.bias is not None else []
            if isinstance(self.normalizer_fn, BatchNorm):
                n = self.normalizer_fn
                rest += [t for t in (n.gamma, n.beta, n.moving_mean, n.moving_variance)
                         if t is not None]
            kt = self.__dict__["_key_ts"] = (w, tuple(rest), w.data_ptr())
        return kt

    def _param_key(self):
        w, rest, _ = self._key_tensors()
        return (w.data_ptr(), w._version) + tuple(t._version for t in rest)

    def _pack_key(self, w):
        return self._param_key() + (tuple(w.shape),)

    def effective_params(self, want_packed=False):
        """(weights HWIO, bias, normalizer still to apply, packed-or-None) with a
        frozen BatchNorm folded in by one fused HIP kernel (d2mi_fold_frozen_bn,
        differentiable w.r.t. weights / bias / gamma / beta).  Cached while
        autograd is off (inference)."""
        norm = self.normalizer_fn
        if not isinstance(norm, BatchNorm):
            return self.weights, self.bias, norm, None
        if not self.weights.is_cuda:
            raise RuntimeError(f"{self.scope}: the FrozenBN fold runs on the GPU (HIP)")
        # constant while autograd is off or nothing in the fold trains (the
        # layers below FREEZE_AT): cached per parameter version
        cacheable = not (torch.is_grad_enabled() and self.fold_trainable())
        group = self.__dict__.get("_fold_group")
        if not cacheable and group is not None:  # (the group checks the versions itself)
            got = group.fetch(self)
            if got is not None:
                return got[0], got[1], None, got[2]
        key = self._param_key()
        if cacheable and getattr(self, "_fold_key", None) == key:
            return self._fold_w, self._fold_b, None, self._fold_p
        w, b, packed = ops.fold_frozen_bn(self.weights, self.bias, norm.gamma, norm.beta,
                                          norm.moving_mean, norm.moving_variance, norm.epsilon,
                                          want_packed)
        if cacheable:
            self._fold_w, self._fold_b, self._fold_p, self._fold_key = w, b, packed, key
        return w, b, None, packed

    def fold_trainable(self):
        norm = self.normalizer_fn
        if self.weights.requires_grad or (self.bias is not None and self.bias.requires_grad):
            return True
        if isinstance(norm, BatchNorm):
            return any(t is not None and t.requires_grad for t in (norm.gamma, norm.beta))
        return False

    def wants_packed(self):
        return (self.impl in ("mfma", "auto") and self.num_groups == 1 and self.rate == 1
                and self.in_channels % 4 == 0)

    def packed_weights(self, w_eff=None):
        group = self.__dict__.get("_pack_group")
        if (group is not None and PackGroup.ENABLED
                and (w_eff is None or w_eff is self.weights)):
            return group.fetch(self)
        w = self.weights if w_eff is None else w_eff
        # the packed tensor's own shape is part of the key: a Cin-padded w_eff
        # (Cin % 4 != 0) packs to [.., Cout, Cin + pad], never to be returned
        # for the layer's own weights (or the other way round)
        key = self._pack_key(w)
        if self._packed is None or self._packed_key != key:
            self._packed = ops.pack_conv_weights(w.detach())
            self._packed_key = key
        return self._packed

    def call_levels(self, inputs):
        """This layer applied to each of ``inputs`` (feature levels sharing the
        layer, as the reference's per-level head calls do), as ONE multi-level
        MFMA launch (ops.conv2d_nhwc_levels) when nothing needs a gradient;
        per-level calls otherwise.  The normalizer / activation follow per
        level (GroupNorm + ReLU fused where it can be)."""
        padded = self.impl == "mfma"  # explicit MFMA: Cin padded to a multiple of 4
        ok = (not torch.is_grad_enabled() and self.impl in ("mfma", "auto") and len(inputs) <= 6
              and all(self._mfma_eligible(x, padded) for x in inputs)
              and not isinstance(self.normalizer_fn, BatchNorm))
        if not ok:
            return [self(x) for x in inputs]
        w, b, norm, packed = self.effective_params(want_packed=True)
        padc = (-self.in_channels) % 4
        if padc:
            inputs = [F.pad(x, (0, padc)) for x in inputs]
            w = F.pad(w, (0, 0, 0, padc))
            packed = None
        if packed is None:
            packed = self.packed_weights(w)
        pads = same_pads(self.kernel_size, self.rate) if self.padding == "SAME" else (0, 0)
        fuse_relu = norm is None and is_relu(self.act_fn)
        ys = ops.conv2d_nhwc_levels(inputs, packed, b, self.stride, pads, relu=fuse_relu)
        if (norm is not None and is_relu(self.act_fn) and hasattr(norm, "fused_ok")
                and all(norm.fused_ok(y) for y in ys)):
            # GroupNorm + ReLU over every level in one set of launches
            return ops.group_norm_levels(ys, norm.num_groups, norm.gamma, norm.beta, norm.epsilon,
                                         relu=True)
        out = []
        for y in ys:
            if norm is not None and is_relu(self.act_fn) and hasattr(norm, "fused_ok") \
                    and norm.fused_ok(y):
                out.append(norm(y, relu=True))
                continue
            if norm is not None:
                y = norm(y)
            if self.act_fn is not None and not fuse_relu:
                y = self.act_fn(y)
            out.append(y)
        return out

    def call(self, inputs, topdown=None, residual=None, relu_after_add=False, final_relu=False,
             relu_input_sole_consumer=False, res_grad_to=None, grad_from=None, pair_grad=None,
             raw=False, join=None, wacc=None):
        """topdown: fused + up2(topdown) (FPN merge); residual: fused + residual;
        relu_after_add: the layer's ReLU runs after those adds; final_relu: an
        extra ReLU after the adds for a layer without activation (the
        bottleneck's relu(conv3(x) + shortcut), blocks.py:143-186)."""
        impl = self.impl
        if impl == "auto":
            impl = "mfma" if self._mfma_eligible(inputs) else "torch"
        w, b, norm, packed = self.effective_params(want_packed=(impl == "mfma"))
        if final_relu:
            if self.act_fn is not None:
                raise ValueError("final_relu is for layers without an activation")
            if impl == "torch":
                return torch.relu_(self.call(inputs, topdown, residual))
        if impl == "mfma":
            if not self._mfma_eligible(inputs, padded=True):
                raise ValueError(f"{self.scope}: shape/device not supported by the MFMA conv "
                                 f"(groups={self.num_groups}, rate={self.rate}, "
                                 f"Cin={self.in_channels}, device={inputs.device})")
            pads = same_pads(self.kernel_size, self.rate) if self.padding == "SAME" else (0, 0)
            fuse_relu = norm is None and (is_relu(self.act_fn) or final_relu)
            relu_after_add = relu_after_add or final_relu
            if (topdown is not None or residual is not None) and fuse_relu and not relu_after_add:
                raise ValueError("relu(conv) + add cannot be fused; use relu_after_add")
            padc = (-self.in_channels) % 4
            if join is not None:
                if padc or not torch.is_grad_enabled():
                    join = None  # (a padded input is another tensor: no join)
                else:
                    join["join"] = True  # the pair members now leave their sum to this layer
            if padc:
                inputs = F.pad(inputs, (0, padc))
                w = F.pad(w, (0, 0, 0, padc))
                packed = None
            if packed is None:
                packed = self.packed_weights(w)
            ret = _ConvMFMAFn.apply(inputs, w, b, packed, self.stride, pads,
                                    fuse_relu, topdown, residual, relu_after_add,
                                    bool(relu_input_sole_consumer), res_grad_to, grad_from,
                                    pair_grad, join, wacc)
            if raw:  # the conv (+ bias) alone: the caller applies the normalizer / activation
                return ret
            if norm is not None and is_relu(self.act_fn) and hasattr(norm, "fused_ok") \
                    and norm.fused_ok(ret):
                return norm(ret, relu=True)  # GroupNorm + ReLU in one HIP pass
            if norm is not None:
                ret = norm(ret)
            if self.act_fn is not None and not fuse_relu:
                ret = self.act_fn(ret)
            if final_relu and not fuse_relu:
                ret = torch.relu(ret)
            return ret
        # torch (channels_last) path: backbone 3x3 convs / the stem.  A symmetric
        # SAME pad is the conv's own zero padding (no padded copy of the input).
        pad = 0
        x = inputs
        if self.padding == "SAME" and self.kernel_size != 1:
            pb, pe = same_pads(self.kernel_size, self.rate)
            if pb == pe:
                pad = pb
            else:
                x = fix_padding(inputs, self.kernel_size, self.padding, self.rate)
        y = F.conv2d(x.permute(0, 3, 1, 2),
                     w.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last), b,
                     stride=self.stride, padding=pad, dilation=self.rate, groups=self.num_groups)
        ret = y.permute(0, 2, 3, 1)
        if norm is not None:
            ret = norm(ret)
        has_add = topdown is not None or residual is not None
        if self.act_fn is not None and not (has_add and relu_after_add):
            ret = self.act_fn(ret)
        if topdown is not None:
            N, H, W, C = ret.shape
            ret = ret + topdown.repeat_interleave(2, 1).repeat_interleave(2, 2)[:, :H, :W]
        if residual is not None:
            ret = ret + residual
        if self.act_fn is not None and has_add and relu_after_add:
            ret = torch.relu_(ret) if is_relu(self.act_fn) else self.act_fn(ret)
        return ret


@add_arg_scope
class ConvTranspose2D(Layer):
    """Transposed conv (convolutional.py:747-893); weights [k, k, out, in].

    For the kernel == stride case of the mask head (2x2, s2) each input pixel
    owns a disjoint 2x2 output block, so the op is one GEMM over
    [pixels, in] x [in, k*k*out]: it runs on the MFMA conv kernel as a 1x1
    conv whose packed weight is the TF kernel itself, followed by a pixel
    shuffle."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding="SAME",
                 use_bias=True, activation=None, normalizer=None, normalizer_params=None,
                 weights_initializer=None, weights_regularizer=None, bias_initializer=None,
                 bias_regularizer=None, variables_collections=None, trainable=True,
                 outputs_collections=None, **kwargs):
        super().__init__(in_channels=in_channels, out_channels=out_channels,
                         kernel_size=kernel_size, stride=stride, padding=padding.upper(),
                         use_bias=use_bias, activation=activation, normalizer=normalizer,
                         normalizer_params=normalizer_params, weights_initializer=weights_initializer,
                         bias_initializer=bias_initializer, trainable=trainable, **kwargs)
        k = kernel_size
        w = torch.empty((k, k, out_channels, in_channels))
        # fans of a transposed kernel: tf computes them on [k, k, out, in]
        (weights_initializer or init.variance_scaling(2.0, distribution="untruncated_normal"))(w)
        self.weights = torch.nn.Parameter(w, requires_grad=trainable)
        self.bias = torch.nn.Parameter(torch.zeros(out_channels), requires_grad=trainable) if use_bias else None
        self.normalizer_fn = None
        if normalizer is not None:
            p = dict(normalizer_params or {})
            p["channels"] = out_channels
            self.normalizer_fn = normalizer(**p)
        self.act_fn = get_activation(activation)

    def call(self, inputs, relu_input_sole_consumer=False):
        k, s = self.kernel_size, self.stride
        N, H, W, C = inputs.shape
        if k == s:  # the mask-head case: MFMA GEMM (raises off-GPU, no CPU fallback)
            wp = self.weights.reshape(1, 1, k * k * self.out_channels, self.in_channels)
            b = self.bias.repeat(k * k) if self.bias is not None else None
            fuse = self.normalizer_fn is None and is_relu(self.act_fn)
            y = _ConvMFMAFn.apply(inputs, wp.permute(0, 1, 3, 2), b, wp.detach().contiguous(), 1,
                                  (0, 0), fuse, None, None, False, bool(relu_input_sole_consumer))
            y = y.reshape(N, H, W, k, k, self.out_channels).permute(0, 1, 3, 2, 4, 5)
            ret = y.reshape(N, H * k, W * k, self.out_channels)
            if self.normalizer_fn is not None:
                ret = self.normalizer_fn(ret)
            if self.act_fn is not None and not fuse:
                ret = self.act_fn(ret)
            return ret
        # general case on torch: conv_transpose2d with TF 'SAME'/'VALID' output size
        w = self.weights.permute(3, 2, 0, 1)  # [in, out, kh, kw]
        y = F.conv_transpose2d(inputs.permute(0, 3, 1, 2), w, self.bias, stride=s)
        OH = H * s + (max(k - s, 0) if self.padding == "VALID" else 0)
        OW = W * s + (max(k - s, 0) if self.padding == "VALID" else 0)
        if self.padding == "SAME":
            ph, pw = max((H - 1) * s + k - OH, 0), max((W - 1) * s + k - OW, 0)
            y = y[:, :, ph // 2: ph // 2 + OH, pw // 2: pw // 2 + OW]
        ret = y.permute(0, 2, 3, 1)
        if self.normalizer_fn is not None:
            ret = self.normalizer_fn(ret)
        if self.act_fn is not None:
            ret = self.act_fn(ret)
        return ret
