"""The training RPN head's output layout (d2mi_rpn_head_gather / _scatter and
d2mi_rpn_proposals_ex): the fused 16-wide 1x1 outputs go straight into the
RPNOutputs concatenation (rpn_outputs.py:346-357) and back, and the proposal
op reads level views of that buffer -- all bit-identical to the slice /
concatenate / contiguous-copy formulation they replace."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def ops():
    from detectron2_tensorflow_amd.layers import ops as o
    return o


SHAPES = [(2, 50, 84, 16), (2, 25, 42, 16), (2, 13, 21, 16), (2, 7, 11, 16)]


def test_rpn_head_gather_and_scatter_match_torch(dev):
    g = torch.Generator().manual_seed(4)
    A = 3
    ys = [torch.randn(s, generator=g).to(dev) for s in SHAPES]
    pl, pd = ops().rpn_head_gather(ys, A)
    N = ys[0].shape[0]
    want_l = torch.cat([y[..., :A].reshape(N, -1) for y in ys], 1)
    want_d = torch.cat([y[..., A:5 * A].reshape(N, -1, 4) for y in ys], 1)
    assert torch.equal(pl, want_l) and torch.equal(pd, want_d)
    gl = torch.randn(pl.shape, generator=g).to(dev)
    gd = torch.randn(pd.shape, generator=g).to(dev)
    for a, b in ((gl, gd), (gl, None), (None, gd)):
        outs = ops().rpn_head_scatter(a, b, [y.shape for y in ys], A)
        off = 0
        for y, o in zip(ys, outs):
            n, h, w, c = y.shape
            hw = h * w
            want = torch.zeros_like(y)
            if a is not None:
                want[..., :A] = a[:, off * A:(off + hw) * A].reshape(n, h, w, A)
            if b is not None:
                want[..., A:5 * A] = b[:, off * A:(off + hw) * A].reshape(n, h, w, 4 * A)
            assert torch.equal(o, want)
            off += hw


def test_rpn_proposals_on_level_views_match_dense(dev):
    g = torch.Generator().manual_seed(5)
    A = 3
    ys = [torch.randn(s, generator=g).to(dev) * 2 for s in SHAPES]
    pl, pd = ops().rpn_head_gather(ys, A)
    views_l, views_d, dense_l, dense_d = [], [], [], []
    off = 0
    for y in ys:
        n, h, w, _ = y.shape
        views_l.append(pl[:, off * A:(off + h * w) * A].view(n, h, w, A))
        views_d.append(pd[:, off * A:(off + h * w) * A].view(n, h, w, 4 * A))
        dense_l.append(y[..., :A].contiguous())
        dense_d.append(y[..., A:5 * A].contiguous())
        off += h * w
    assert not views_l[1].is_contiguous()
    strides = [16, 32, 64, 128]
    cells = [torch.tensor([[-22.6, -11.3, 22.6, 11.3], [-16.0, -16.0, 16.0, 16.0],
                           [-11.3, -22.6, 11.3, 22.6]]) * (s / 16) for s in strides]
    image_hw = torch.tensor([[800, 1333], [760, 1300]], dtype=torch.int32, device=dev)
    kw = dict(strides=strides, cell_anchors=cells, image_hw=image_hw, pre_nms_topk=1000,
              post_nms_topk=1000, nms_thresh=0.7, min_box_side_len=0.0)
    a = ops().rpn_proposals(views_l, views_d, **kw)
    b = ops().rpn_proposals(dense_l, dense_d, **kw)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
