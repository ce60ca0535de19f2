"""BatchNorm training kernels (csrc/bn.hip) against a torch float64 restatement of
Keras' BatchNormalization in training mode (the pix2pix / SR blocks,
pix2pix.py:110-142, srgan.py:129-185): batch statistics with the biased variance,
the moving averages updated with the unbiased one (moving -= (moving - value) *
(1 - momentum)), the fused activation, and the backward's dy / dgamma / dbeta.

Covers several segments (independent statistics per segment, the moving
averages updated one segment after the other), the row-chunk partial passes at
the SR family's size (18 432 rows -> 256 chunks), wide channel counts (512),
channel counts off the finalize block width (96), the scalar path (C = 3),
pixel strides and the beta = 1 accumulation of dgamma / dbeta.  Tolerances:
fp32 kernels vs fp64, 2e-5 of the output scale (5e-5 for the backward sums)."""
import pytest
import torch

gpu = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # (name, segments, rows per segment, C, act, pixel stride padding)
    ("srgan.res", 1, 18432, 64, "none", 0),
    ("seg2.lrelu", 2, 4096, 32, "lrelu", 0),
    ("deep.c512", 1, 64, 512, "relu", 0),
    ("c96.strided", 1, 1000, 96, "lrelu", 4),
    ("c3.scalar", 1, 37, 3, "none", 0),
    ("seg2.c256", 2, 2048, 256, "relu", 0),
    # a ragged last chunk, 4 and 1024 channels, two large segments (pix2pix down3)
    ("ragged", 1, 9001, 64, "lrelu", 0),
    ("c4", 1, 20000, 4, "relu", 0),
    ("c1024", 1, 300, 1024, "none", 0),
    ("seg2.down3", 2, 16384, 256, "lrelu", 0),
]


def _act(t, act, alpha):
    if act == "relu":
        return torch.relu(t)
    if act == "lrelu":
        return torch.where(t > 0, t, alpha * t)
    return t


def _ref(y, g, b, dz, mm, mv, S, act, alpha, momentum, eps):
    """fp64 forward + backward per segment; moving statistics updated segment by segment."""
    M = y.shape[0] // S
    zs, dys = [], []
    dg = torch.zeros_like(g)
    db = torch.zeros_like(b)
    mm, mv = mm.clone(), mv.clone()
    means, invs = [], []
    for s in range(S):
        ys = y[s * M:(s + 1) * M].clone().requires_grad_()
        gs, bs = g.clone().requires_grad_(), b.clone().requires_grad_()
        mean = ys.mean(0)
        var = ys.var(0, unbiased=False)
        inv = 1.0 / torch.sqrt(var + eps)
        z = _act((ys - mean) * inv * gs + bs, act, alpha)
        z.backward(dz[s * M:(s + 1) * M])
        zs.append(z.detach())
        dys.append(ys.grad)
        dg += gs.grad
        db += bs.grad
        unb = ys.detach().var(0, unbiased=True) if M > 1 else var.detach()
        mm -= (mm - mean.detach()) * (1 - momentum)
        mv -= (mv - unb) * (1 - momentum)
        means.append(mean.detach())
        invs.append(inv.detach())
    return torch.cat(zs), torch.cat(dys), dg, db, mm, mv, torch.stack(means), torch.stack(invs)


def _close(got, ref, what, rel=2e-5):
    g = got.double().cpu()
    err = float((g - ref).abs().max())
    scale = max(float(ref.abs().max()), 1e-6)
    assert err <= rel * scale, f"{what}: max-abs {err:.3e} vs scale {scale:.3e}"


@gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_bn_train_matches_fp64(case):
    from dgan import ops
    name, S, M, C, act, pad = case
    torch.manual_seed(sum(map(ord, name)))
    alpha, momentum, eps = 0.2, 0.99, 1e-3
    R = S * M
    y64 = (torch.randn(R, C, dtype=torch.float64) * 1.7 + 0.4)
    dz64 = torch.randn(R, C, dtype=torch.float64)
    g64 = 1 + 0.2 * torch.randn(C, dtype=torch.float64)
    b64 = 0.1 * torch.randn(C, dtype=torch.float64)
    mm64 = 0.05 * torch.randn(C, dtype=torch.float64)
    mv64 = 1 + 0.1 * torch.rand(C, dtype=torch.float64)
    # the kernels see the fp32-rounded inputs: the reference starts from the same values
    y64, dz64, g64, b64, mm64, mv64 = (t.float().double() for t in (y64, dz64, g64, b64, mm64, mv64))
    z_r, dy_r, dg_r, db_r, mm_r, mv_r, mean_r, inv_r = _ref(y64, g64, b64, dz64, mm64, mv64, S, act, alpha,
                                                            momentum, eps)
    big = torch.zeros(R, C + pad, device=DEV)
    big[:, :C] = y64.float().to(DEV)
    y = big[:, :C].view(1, 1, R, C)   # (a pixel stride of C + pad when padded)
    z = torch.empty(1, 1, R, C, device=DEV)
    g, b = g64.float().to(DEV), b64.float().to(DEV)
    mm, mv = mm64.float().to(DEV), mv64.float().to(DEV)
    mean, inv = torch.empty(S, C, device=DEV), torch.empty(S, C, device=DEV)
    ops.bn_fwd_train(y, g, b, mean, inv, mm, mv, z, act=act, alpha=alpha, momentum=momentum, eps=eps, segments=S)
    dz = dz64.float().to(DEV).view(1, 1, R, C)
    dy = torch.empty(1, 1, R, C, device=DEV)
    dg = torch.full((C,), 0.5, device=DEV)
    db = torch.full((C,), -0.25, device=DEV)
    ops.bn_bwd(dz, z, y, g, mean, inv, dy, dg, db, act=act, alpha=alpha, beta=1.0, segments=S)
    torch.cuda.synchronize()
    _close(z.view(R, C), z_r, "z")
    _close(mean, mean_r, "mean")
    _close(inv, inv_r, "invstd")
    _close(mm, mm_r, "moving mean", rel=1e-5)
    _close(mv, mv_r, "moving variance", rel=1e-5)
    _close(dy.view(R, C), dy_r, "dy", rel=5e-5)
    _close(dg, dg_r + 0.5, "dgamma (beta = 1 accumulation)", rel=5e-5)
    _close(db, db_r - 0.25, "dbeta (beta = 1 accumulation)", rel=5e-5)
    # deterministic: the same call again gives the same bits (fixed chunks, fixed-order folds)
    z2 = torch.empty_like(z)
    mean2, inv2 = torch.empty_like(mean), torch.empty_like(inv)
    mm2, mv2 = mm64.float().to(DEV), mv64.float().to(DEV)
    ops.bn_fwd_train(y, g, b, mean2, inv2, mm2, mv2, z2, act=act, alpha=alpha, momentum=momentum, eps=eps,
                     segments=S)
    dy2 = torch.empty_like(dy)
    dg2, db2 = torch.full((C,), 0.5, device=DEV), torch.full((C,), -0.25, device=DEV)
    ops.bn_bwd(dz, z2, y, g, mean2, inv2, dy2, dg2, db2, act=act, alpha=alpha, beta=1.0, segments=S)
    torch.cuda.synchronize()
    for a, b_, what in ((z, z2, "z"), (mm, mm2, "moving mean"), (mv, mv2, "moving var"), (dy, dy2, "dy"),
                        (dg, dg2, "dgamma"), (db, db2, "dbeta")):
        assert torch.equal(a, b_), f"{what} differs between two identical calls"



@gpu
@pytest.mark.parametrize("act", ["lrelu", "relu"])
@pytest.mark.parametrize("planes", [False, True])
def test_bn_bwd_act_from_y_equals_from_z(act, planes):
    """dg_bn_bwd_seg_r (act'(z) from the sign of y * scale + shift, z not read) gives the bits
    of dg_bn_bwd_seg_x reading the forward's z: dy, dgamma, dbeta and the fp16x3 dy planes with
    their bound -- on two segments whose pre-activations crowd around 0 (beta 0, y within a
    few ulps of the mean in a third of the channels), where a sign differing by one rounding
    would show."""
    from dgan import ops
    torch.manual_seed(7 + planes)
    S, M, C = 2, 3000, 96
    R = S * M
    y = torch.randn(R, C) * 1.3 + 0.2
    y[:, ::3] = 0.5 + 1e-6 * torch.randn(R, (C + 2) // 3)   # t = (y - mean) * scale ~ rounding noise
    y = y.to(DEV).view(1, 1, R, C)
    g = (1 + 0.2 * torch.randn(C)).to(DEV)
    b = torch.zeros(C, device=DEV)
    b[1::3] = 0.1 * torch.randn((C + 1) // 3).to(DEV)
    mm, mv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    mean, inv = torch.empty(S, C, device=DEV), torch.empty(S, C, device=DEV)
    z = torch.empty(1, 1, R, C, device=DEV)
    ops.bn_fwd_train(y, g, b, mean, inv, mm, mv, z, act=act, alpha=0.3, segments=S)
    dz = torch.randn(1, 1, R, C).to(DEV)
    out = []
    for zz, off in ((z, None), (None, b)):
        dy = torch.empty(1, 1, R, C, device=DEV)
        dg, db = torch.full((C,), 0.5, device=DEV), torch.full((C,), -0.25, device=DEV)
        pl = torch.zeros(R * C * 4, dtype=torch.uint8, device=DEV) if planes else None
        bnd = ops.max_slot(device=DEV) if planes else None
        ops.bn_bwd(dz, zz, y, g, mean, inv, dy, dg, db, act=act, alpha=0.3, beta=1.0, segments=S,
                   dy_planes=pl, dy_bound=bnd, offset=off)
        out.append((dy, dg, db, pl, bnd))
    torch.cuda.synchronize()
    near0 = (z.view(R, C)[:, ::3].abs() < 1e-4).float().mean().item()
    assert near0 > 0.5, f"the crowded channels sit near 0 ({near0:.2f})"
    for a, b_, what in zip(out[0], out[1], ("dy", "dgamma", "dbeta", "dy planes", "dy bound")):
        if a is not None:
            assert torch.equal(a, b_), f"{what}: recomputed act' differs from the one read from z"
