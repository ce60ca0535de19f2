"""Producer-written bf16x6 planes of the BatchNorm kernels
(include/dgan.h dg_bn_fwd_train_pl / dg_bn_bwd_pl).

The planes a BN pass writes beside its fp32 output must be byte-identical to
the planes the consuming conv would split from that output itself
(dg_conv_planes_t, layout r*3C + (c/16)*48 + 16p + c%16), including a column
slice of a wider concat consumer (the U-Net skip connections)."""
import pytest
import torch

from dgan import ops

gpu = pytest.mark.gpu


def _rand(shape, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).cuda()


def _split_by_conv(t, tensor_bit):
    """The planes a bf16x6 conv splits from t (as its x, or as its dy)."""
    N, H, W, C = t.shape
    if tensor_bit == ops.TENSOR_X:
        d = ops.ConvDesc(N, H, W, C, 64, 4, 2, "same", math="bf16x6")
        P = ops.ConvPlanes.for_desc(d, x=True, w=True)
        w = _rand(d.weight_shape, 9, 0.05)
        d.fwd(t, w, torch.empty(d.out_shape, device="cuda"), planes=P)
        return P.x.buf
    d = ops.ConvDesc(N, 2 * H, 2 * W, 64, C, 4, 2, "same", math="bf16x6")
    P = ops.ConvPlanes.for_desc(d, dy=True)
    x = _rand((N, 2 * H, 2 * W, 64), 8)
    d.bwd_filter(x, t, torch.empty(d.weight_shape, device="cuda"), planes=P)
    return P.dy.buf


def _bn_state(C):
    return dict(gamma=_rand((C,), 3, 0.1) + 1.0, beta=_rand((C,), 4, 0.1),
                mean=torch.empty(C, device="cuda"), inv=torch.empty(C, device="cuda"),
                mm=torch.zeros(C, device="cuda"), mv=torch.ones(C, device="cuda"))


@pytest.fixture(autouse=True)
def _x6_plans(monkeypatch):
    # the reference splits come from bf16x6 plans (the planner would keep
    # these small GEMMs on the fp32 kernel, which reads no planes)
    monkeypatch.setenv("DG_FORCE_X6CFG", "0")


@gpu
@pytest.mark.parametrize("act", ["lrelu", "relu"])
def test_bn_forward_planes_match_split(act):
    N, H, W, C = 4, 16, 16, 64
    y = _rand((N, H, W, C), 1)
    s = _bn_state(C)
    rows = N * H * W
    full = torch.zeros(rows * 6 * C, dtype=torch.uint8, device="cuda")
    # the same output as the second half (columns C..2C) of a 2C-wide concat consumer
    cat = torch.zeros(rows * 6 * 2 * C, dtype=torch.uint8, device="cuda")
    z = torch.empty_like(y)
    ops.bn_fwd_train(y, s["gamma"], s["beta"], s["mean"], s["inv"], s["mm"], s["mv"], z, act=act,
                     z_planes=[(full, C, 0), (cat, 2 * C, C)])
    z_ref = torch.empty_like(y)
    s2 = _bn_state(C)
    ops.bn_fwd_train(y, s2["gamma"], s2["beta"], s2["mean"], s2["inv"], s2["mm"], s2["mv"], z_ref, act=act)
    torch.cuda.synchronize()
    assert torch.equal(z, z_ref)
    ref = _split_by_conv(z, ops.TENSOR_X)
    assert torch.equal(full, ref[:full.numel()])
    # column slice: per row, the second C-channel half of the 2C-wide planes
    got = cat.view(rows, 2 * C // 16, 96)[:, C // 16:, :].reshape(-1)
    assert torch.equal(got, ref[:full.numel()])
    assert torch.count_nonzero(cat.view(rows, 2 * C // 16, 96)[:, :C // 16, :]) == 0


@gpu
def test_bn_backward_planes_match_split():
    N, H, W, C = 4, 16, 16, 128
    y = _rand((N, H, W, C), 1)
    s = _bn_state(C)
    z = torch.empty_like(y)
    ops.bn_fwd_train(y, s["gamma"], s["beta"], s["mean"], s["inv"], s["mm"], s["mv"], z, act="lrelu")
    dz = _rand((N, H, W, C), 2)
    dy = torch.empty_like(y)
    dyp = torch.zeros(N * H * W * 6 * C, dtype=torch.uint8, device="cuda")
    dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    ops.bn_bwd(dz, z, y, s["gamma"], s["mean"], s["inv"], dy, dg, db, act="lrelu", dy_planes=dyp)
    dy_ref = torch.empty_like(y)
    ops.bn_bwd(dz, z, y, s["gamma"], s["mean"], s["inv"], dy_ref, torch.empty_like(dg), torch.empty_like(db),
               act="lrelu")
    torch.cuda.synchronize()
    assert torch.equal(dy, dy_ref)
    ref = _split_by_conv(dy, ops.TENSOR_DY)
    assert torch.equal(dyp, ref[:dyp.numel()])
