"""Max pool fused into the conv's forward epilogue (dg_conv_fwd_pool) and its
index-byte backward (dg_maxpool2_bwd_idx), against the unfused pair
(dg_conv_fwd_pl + dg_maxpool2_fwd_pl / dg_maxpool2_bwd_pl) that the VGG19
content loss ran before (keras VGG19 blockN_conv -> blockN_pool, as built by
pix2pix.py:53-67 and srgan.py:70-76).

The fused epilogue applies the same bias + activation to the same fp32
accumulators and picks the same first maximum, so every output is compared
bit for bit: the pooled values, their bf16x6 planes, the argmax (against the
window of the unfused full-size activation) and the routed gradient with its
planes."""
import pytest
import torch

from dgan import ops
from dgan._lib import DGError

gpu = pytest.mark.gpu

# N, H, W, Cin, Cout, act: the halo kernel's two tile widths (Cout 64 / 128),
# ReLU (VGG19) and LeakyReLU; sizes with one split (pool_fusable)
CASES = [
    (16, 64, 64, 32, 64, "relu"),
    (16, 64, 64, 32, 128, "relu"),
    (8, 64, 64, 32, 128, "lrelu"),
]


def _rand(shape, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).cuda()


def _bytes(pb, n):
    return pb.buf[:n].clone()


@gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:5])) + c[5])
def test_fused_pool_matches_conv_then_pool(case):
    N, H, W, Cin, Cout, act = case
    d = ops.ConvDesc(N, H, W, Cin, Cout, 3, 1, "same", math="bf16x6")
    assert d.pool_fusable(act)
    x = _rand((N, H, W, Cin), 1)
    w = _rand(d.weight_shape, 2, 0.05)
    b = _rand((Cout,), 3, 0.1)
    ws = ops.Workspace()
    # unfused: full-size activation, then the pool (values + planes of the pooled output)
    y = torch.empty(d.out_shape, device="cuda")
    d.fwd(x, w, y, bias=b, act=act, ws=ws)
    py0 = torch.empty((N, H // 2, W // 2, Cout), device="cuda")
    nb = N * (H // 2) * (W // 2) * Cout * 6
    pl0 = ops.PlaneBuf(nb)
    ops.maxpool2_fwd(y, py0, planes_out=pl0)
    # fused
    py1 = torch.full_like(py0, float("nan"))
    pl1 = ops.PlaneBuf(nb)
    idx = torch.empty((N, H // 2, W // 2, Cout), dtype=torch.uint8, device="cuda")
    d.fwd_pool(x, w, idx, bias=b, act=act, pool_y=py1, ws=ws, pool_planes=pl1)
    torch.cuda.synchronize()
    assert torch.equal(py0.view(torch.int32), py1.view(torch.int32))
    assert torch.equal(_bytes(pl0, nb), _bytes(pl1, nb))
    # argmax byte == first maximum of the unfused window; bit 2 == pooled > 0
    win = y.reshape(N, H // 2, 2, W // 2, 2, Cout).permute(0, 1, 3, 5, 2, 4).reshape(N, H // 2, W // 2, Cout, 4)
    first = win.argmax(dim=-1)   # torch.argmax returns the first maximal index
    ib = idx.long()
    assert torch.equal(ib & 3, first)
    assert torch.equal((ib & 4) != 0, py0 > 0)
    # a decisive test: the windows are not all ties at 0
    assert (first != 0).float().mean() > 0.3

    # backward: routed gradient and its planes, fp32 dx kept or dropped
    dy = _rand((N, H // 2, W // 2, Cout), 4)
    dx0 = torch.empty_like(y)
    nbx = N * H * W * Cout * 6
    g0 = ops.PlaneBuf(nbx)
    ops.maxpool2_bwd(y, dy, dx0, act=act, alpha=0.3, planes_out=g0)
    dx1 = torch.full_like(dx0, float("nan"))
    g1 = ops.PlaneBuf(nbx)
    ops.maxpool2_bwd_idx(idx, dy, dx1, Cout, H, W, act=act, alpha=0.3, planes_out=g1)
    g2 = ops.PlaneBuf(nbx)
    ops.maxpool2_bwd_idx(idx, dy, None, Cout, H, W, act=act, alpha=0.3, planes_out=g2)
    torch.cuda.synchronize()
    assert torch.equal(dx0.view(torch.int32), dx1.view(torch.int32))
    assert torch.equal(_bytes(g0, nbx), _bytes(g1, nbx))
    assert torch.equal(_bytes(g0, nbx), _bytes(g2, nbx))


@gpu
def test_fused_pool_refuses_ineligible_plans():
    # 3x3 s1 on 12 x 12 (not whole 8 x 16 patches) and a stride-2 4x4 conv (no halo plan)
    for args in ((4, 12, 12, 64, 64, 3, 1, "same"), (8, 64, 64, 64, 128, 4, 2, "same")):
        d = ops.ConvDesc(*args, math="bf16x6")
        assert not d.pool_fusable("relu")
        x = torch.zeros((args[0], args[1], args[2], args[3]), device="cuda")
        w = torch.zeros(d.weight_shape, device="cuda")
        N, Ho, Wo, Co = d.out_shape
        idx = torch.empty((N, Ho // 2, Wo // 2, Co), dtype=torch.uint8, device="cuda")
        py = torch.empty((N, Ho // 2, Wo // 2, Co), device="cuda")
        with pytest.raises(DGError):
            d.fwd_pool(x, w, idx, act="relu", pool_y=py, ws=ops.Workspace())
    d = ops.ConvDesc(16, 64, 64, 32, 64, 3, 1, "same", math="bf16x6")
    assert not d.pool_fusable("tanh")


@gpu
@pytest.mark.parametrize("shape", [(8, 64, 64, 64, 64), (16, 16, 16, 512, 512)], ids=["b1c2like", "b5like_splitk"])
def test_planes_only_forward_and_plane_mask(shape):
    """A conv -> conv chain without the fp32 activation (the frozen VGG19's
    planes-only layers): the producer's planes-only forward writes the same
    planes as its full forward, and the consumer's input gradient masked by
    the planes' sign (dg_conv_bwd_data_xmask) equals the fp32-masked one."""
    N, H, W, C, Co = shape
    d0 = ops.ConvDesc(N, H, W, C, C, 3, 1, "same", math="bf16x6")   # producer
    d1 = ops.ConvDesc(N, H, W, C, Co, 3, 1, "same", math="bf16x6")  # consumer
    x = _rand((N, H, W, C), 11)
    w0 = _rand(d0.weight_shape, 12, 0.05)
    w1 = _rand(d1.weight_shape, 13, 0.05)
    ws = ops.Workspace()
    nb = N * H * W * C * 6
    # full forward (fp32 + the consumer's planes) vs planes only
    z = torch.empty(d0.out_shape, device="cuda")
    P0 = ops.ConvPlanes(fwd_out=ops.PlaneBuf(nb))
    d0.fwd(x, w0, z, act="relu", ws=ws, planes=P0)
    P1 = ops.ConvPlanes(fwd_out=ops.PlaneBuf(nb))
    d0.fwd(x, w0, None, act="relu", ws=ws, planes=P1)
    torch.cuda.synchronize()
    assert torch.equal(_bytes(P0.fwd_out, nb), _bytes(P1.fwd_out, nb))
    # consumer's input gradient: fp32 mask vs plane mask (x planes = the producer's output planes)
    dy = _rand(d1.out_shape, 14)
    dx0 = torch.empty_like(z)
    d1.bwd_data_masked(dy, w1, dx0, z, "relu", ws=ws)
    dx1 = torch.full_like(z, float("nan"))
    Q = ops.ConvPlanes(x=P1.fwd_out)
    Q.x.ready = True
    d1.bwd_data_xmask(dy, w1, dx1, "relu", ws=ws, planes=Q)
    torch.cuda.synchronize()
    assert (z > 0).float().mean() > 0.2 and (z <= 0).float().mean() > 0.2
    assert torch.equal(dx0.view(torch.int32), dx1.view(torch.int32))
