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


@gpu
@pytest.mark.parametrize("halo", [True, False])
def test_output_planes_feed_the_next_conv(halo, monkeypatch):
    """dg_conv_planes_t.out: a conv writes the planes of its output (fwd) or
    input gradient (bwd_data) for the next conv, which then reads them
    instead of splitting -- results bit-identical to splitting (VGG19 chains,
    GraphPlan fed_x / fed_dy).  Covers the halo kernel (3x3 s1) and the
    generic kernel + split-K reduce (4x4 s2)."""
    monkeypatch.setenv("DG_FORCE_X6CFG", "0")  # bf16x6 plans at these small sizes
    if halo:
        d1 = ops.ConvDesc(4, 32, 32, 64, 64, 3, 1, "same", math="bf16x6")
        d2 = ops.ConvDesc(4, 32, 32, 64, 128, 3, 1, "same", math="bf16x6")
    else:
        d1 = ops.ConvDesc(8, 32, 32, 64, 128, 4, 2, "same", math="bf16x6")
        d2 = ops.ConvDesc(8, 16, 16, 128, 256, 4, 2, "same", math="bf16x6")
    assert d2.plane_mask[ops.OP_FWD] & ops.TENSOR_X and d1.plane_mask[ops.OP_BWD_DATA] & ops.TENSOR_DY
    x = _rand((d1.N, d1.H, d1.W, d1.Cin), 11)
    w1 = _rand(d1.weight_shape, 12) * 0.05
    w2 = _rand(d2.weight_shape, 13) * 0.05
    dz = _rand(d2.out_shape, 14)
    ws = ops.Workspace()
    # reference: every op splits its own operands
    y0 = torch.empty(d1.out_shape, device="cuda")
    z0 = torch.empty(d2.out_shape, device="cuda")
    dy0 = torch.empty_like(y0)
    dx0 = torch.empty_like(x)
    d1.fwd(x, w1, y0, act="relu", ws=ws)
    d2.fwd(y0, w2, z0, ws=ws)
    d2.bwd_data_masked(dz, w2, dy0, y0, "relu", ws=ws)
    d1.bwd_data(dy0, w1, dx0, ws=ws)
    # fed: d1.fwd writes d2's x planes, d2.bwd_data writes d1's dy planes
    p2x = ops.PlaneBuf(d2.plane_bytes(ops.TENSOR_X))
    p1dy = ops.PlaneBuf(d1.plane_bytes(ops.TENSOR_DY))
    y1 = torch.empty_like(y0)
    z1 = torch.full_like(z0, float("nan"))
    dy1 = torch.empty_like(dy0)
    dx1 = torch.full_like(dx0, float("nan"))
    d1.fwd(x, w1, y1, act="relu", ws=ws, planes=ops.ConvPlanes(fwd_out=p2x))
    assert p2x.ready
    keep = y1.clone()
    y1.fill_(float("nan"))     # d2 must read the planes, not the fp32 tensor
    d2.fwd(y1, w2, z1, ws=ws, planes=ops.ConvPlanes(x=p2x))
    y1.copy_(keep)
    d2.bwd_data_masked(dz, w2, dy1, y1, "relu", ws=ws, planes=ops.ConvPlanes(bwd_out=p1dy))
    assert p1dy.ready
    keep = dy1.clone()
    dy1.fill_(float("nan"))
    d1.bwd_data(dy1, w1, dx1, ws=ws, planes=ops.ConvPlanes(dy=p1dy))
    torch.cuda.synchronize()
    assert torch.equal(z0, z1)
    assert torch.equal(dy0, keep)
    assert torch.equal(dx0, dx1)
