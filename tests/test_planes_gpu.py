"""Caller-held bf16x6 operand planes (include/dgan.h dg_conv_planes_t).

A conv op that reads planes another op split (ready bits) must give exactly
the result of the op splitting its own operands: the planes are a pure
function of the tensor, so the outputs are bit-identical.  Covers both
layer kinds (Conv2D, Conv2DTranspose) and all three ops, in the order the
training step uses them (fwd fills X and W; bwd_filter fills DY and reuses
X; bwd_data reuses DY and W)."""
import pytest
import torch

from dgan import ops

gpu = pytest.mark.gpu

SHAPES = [
    # N, H, W, Cin, Cout, k, s, padding, transpose
    # (shapes whose three plans all run on the bf16x6 kernel; the planner
    # keeps small GEMMs on the fp32 kernel, where planes do not apply)
    (16, 64, 64, 64, 128, 4, 2, "same", False),        # U-Net down block
    (8, 32, 32, 128, 64, 4, 2, "same", True),          # U-Net up block
    (8, 24, 24, 128, 128, 3, 1, "same", False),        # VGG / SR 3x3
    (2, 33, 33, 128, 128, 4, 1, (1, 1, 1, 1), False),  # PatchGAN down4-like, odd size
]


def _rand(shape, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(shape, generator=g).cuda()


def _id(s):
    return "x".join(map(str, s[:7])) + ("T" if s[8] else "")


@gpu
@pytest.mark.parametrize("shape", SHAPES, ids=_id)
def test_planes_reuse_is_bit_identical(shape):
    N, H, W, Cin, Cout, k, s, pad, tr = shape
    d = ops.ConvDesc(N, H, W, Cin, Cout, k, s, pad, transpose=tr, math="bf16x6")
    mask = d.plane_mask
    assert mask[ops.OP_FWD] and mask[ops.OP_BWD_DATA] and mask[ops.OP_BWD_FILTER], mask
    x = _rand((N, H, W, Cin), 1)
    w = _rand(d.weight_shape, 2) * 0.05
    dy = _rand(d.out_shape, 3)
    ws = ops.Workspace()
    # reference: every op splits its own operands into the workspace
    y0 = torch.empty(d.out_shape, device="cuda")
    dx0 = torch.empty_like(x)
    dw0 = torch.empty_like(w)
    d.fwd(x, w, y0, ws=ws)
    d.bwd_filter(x, dy, dw0, ws=ws)
    d.bwd_data(dy, w, dx0, ws=ws)
    # planes: fwd fills X and W, bwd_filter fills DY and reuses X, bwd_data reuses DY and W
    P = ops.ConvPlanes.for_desc(d, x=True, w=True, dy=True)
    y1 = torch.full_like(y0, float("nan"))
    dx1 = torch.full_like(dx0, float("nan"))
    dw1 = torch.full_like(dw0, float("nan"))
    d.fwd(x, w, y1, ws=ws, planes=P)
    assert P.ready == ops.TENSOR_X | ops.TENSOR_W
    # scribble over the fp32 operands: a reusing op must read the planes only
    keep = (x.clone(), w.clone(), dy.clone())
    x.fill_(float("nan"))
    d.bwd_filter(x, dy, dw1, ws=ws, planes=P)
    assert P.ready == ops.TENSOR_X | ops.TENSOR_W | ops.TENSOR_DY
    w.fill_(float("nan"))
    dy.fill_(float("nan"))
    d.bwd_data(dy, w, dx1, ws=ws, planes=P)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert torch.equal(dw0, dw1)
    assert torch.equal(dx0, dx1)
    # invalidation: cleared ready bits re-split from the (restored) fp32 tensors
    x.copy_(keep[0])
    w.copy_(keep[1])
    dy.copy_(keep[2])
    P.invalidate(ops.TENSOR_X | ops.TENSOR_W | ops.TENSOR_DY)
    P.dy.buf.zero_()
    dx1.fill_(float("nan"))
    d.bwd_data(dy, w, dx1, ws=ws, planes=P)
    torch.cuda.synchronize()
    assert torch.equal(dx0, dx1)


@gpu
def test_planes_ignored_by_fp32_and_narrow_plans():
    # fp32 math and a narrow (Cout=1) layer take no planes: their masks are 0
    # and passing a ConvPlanes changes nothing
    d1 = ops.ConvDesc(2, 16, 16, 64, 1, 4, 1, (1, 1, 1, 1), math="bf16x6")
    assert d1.plane_mask[ops.OP_FWD] == 0
    d32 = ops.ConvDesc(2, 16, 16, 64, 64, 3, 1, "same", math="fp32")
    assert d32.plane_mask == [0, 0, 0]
    x = _rand((2, 16, 16, 64), 5)
    w = _rand(d32.weight_shape, 6) * 0.05
    P = ops.ConvPlanes(x=ops.PlaneBuf(16))
    y0 = torch.empty(d32.out_shape, device="cuda")
    y1 = torch.empty_like(y0)
    d32.fwd(x, w, y0)
    d32.fwd(x, w, y1, planes=P)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert P.ready == 0
