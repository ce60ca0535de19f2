"""One-launch BatchNorm for small layers (csrc/bn.hip k_bn_fwd_small /
k_bn_bwd_small: the deep U-Net layers, pix2pix.py:110-142) against the
chunked partial -> finalize -> apply path (DG_BN_SMALL_MAX=0) and a float64
torch restatement of Keras' training-mode BatchNormalization (biased variance
for normalisation, unbiased into the moving variance, eps 1e-3, momentum 0.99,
segments = independent calls applied in order)."""
import os

import pytest
import torch

from dgan import ops

gpu = pytest.mark.gpu

CASES = [
    # (segments, rows per segment, channels, act, dropout)
    (2, 16 * 2 * 2, 512, "lrelu", 0.0),    # down7 of the batched G(x) / G(y) pass
    (2, 16 * 8 * 8, 512, "relu", 0.5),     # up3 (dropout + ReLU)
    (1, 300, 64, "none", 0.0),             # ragged rows, one segment
]


def _ref_fwd(y, gamma, beta, mm, mv, S, act, eps=1e-3, mom=0.99):
    yd = y.double().cpu().reshape(S, -1, y.shape[-1])
    gamma, beta = gamma.double().cpu(), beta.double().cpu()
    z, means, invs = [], [], []
    mm, mv = mm.double().clone(), mv.double().clone()
    for s in range(S):
        mu = yd[s].mean(0)
        var = yd[s].var(0, unbiased=False)
        inv = 1.0 / torch.sqrt(var + eps)
        t = (yd[s] - mu) * inv * gamma.double() + beta.double()
        z.append(t)
        means.append(mu)
        invs.append(inv)
        n = yd[s].shape[0]
        mm = mm * mom + mu * (1 - mom)
        mv = mv * mom + var * n / (n - 1) * (1 - mom)
    return torch.cat(z), torch.stack(means), torch.stack(invs), mm, mv


def _run(y, gamma, beta, S, act, rate, small, seed=7):
    C = y.shape[-1]
    M = y.shape[0] // S
    mm = torch.full((C,), 0.1, device="cuda")
    mv = torch.full((C,), 0.9, device="cuda")
    sm, si = torch.empty(S, C, device="cuda"), torch.empty(S, C, device="cuda")
    z = torch.empty_like(y)
    old = os.environ.get("DG_BN_SMALL_MAX")
    os.environ["DG_BN_SMALL_MAX"] = str(1 << 30) if small else "0"
    try:
        ops.bn_fwd_train(y.view(S * M, 1, 1, C), gamma, beta, sm, si, mm, mv, z.view(S * M, 1, 1, C), act=act,
                         drop_rate=rate, drop_seed=seed, segments=S, drop_seed_stride=101)
        dz = torch.randn_like(y)
        dy = torch.empty_like(y)
        dg, db = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        ops.bn_bwd(dz.view(S * M, 1, 1, C), z.view(S * M, 1, 1, C), y.view(S * M, 1, 1, C), gamma, sm, si,
                   dy.view(S * M, 1, 1, C), dg, db, act=act, drop_rate=rate, segments=S)
    finally:
        os.environ.pop("DG_BN_SMALL_MAX", None)
        if old is not None:
            os.environ["DG_BN_SMALL_MAX"] = old
    torch.cuda.synchronize()
    return dict(z=z, mean=sm, inv=si, mm=mm, mv=mv, dy=dy, dg=dg, db=db)


@gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"S{c[0]}M{c[1]}C{c[2]}{c[3]}{c[4]}")
def test_bn_small_path_matches_chunked_and_fp64(case):
    S, M, C, act, rate = case
    torch.manual_seed(0)
    y = (torch.randn(S * M, C) * 2.0 + 0.5).cuda()
    gamma = (torch.rand(C) + 0.5).cuda()
    beta = (torch.randn(C) * 0.1).cuda()
    torch.manual_seed(1)
    a = _run(y, gamma, beta, S, act, rate, small=True)
    torch.manual_seed(1)
    b = _run(y, gamma, beta, S, act, rate, small=False)
    # the two paths sum in different orders: fp32 rounding apart
    for k in a:
        assert torch.allclose(a[k], b[k], rtol=2e-5, atol=2e-5), (k, (a[k] - b[k]).abs().max().item())
    # statistics and moving averages against float64 (no activation / dropout in these)
    _, mu, inv, mm, mv = _ref_fwd(y, gamma, beta, torch.full((C,), 0.1), torch.full((C,), 0.9), S, act)
    assert torch.allclose(a["mean"].double().cpu(), mu, rtol=1e-5, atol=1e-5)
    assert torch.allclose(a["inv"].double().cpu(), inv, rtol=1e-5, atol=1e-5)
    assert torch.allclose(a["mm"].double().cpu(), mm, rtol=1e-5, atol=1e-6)
    assert torch.allclose(a["mv"].double().cpu(), mv, rtol=1e-5, atol=1e-6)
