"""BatchNorm forward statistics written by the producing conv's GEMM epilogue
(include/dgan.h dg_conv_fwd_bnstats + dg_bn_fwd_train_stats; the BN sites
pix2pix.py:115+119, :130+135, :207+211 and srgan.py:129-185).

Against a torch fp64 reference of Keras' training-mode BatchNormalization on
the same conv output: per segment mean / biased variance (normalisation),
moving averages with the unbiased variance, then act(BN(y)).  The fused path
must also leave the conv output itself bit-identical to the plain forward, and
match the statistics-pass path (dg_bn_fwd_train_seg) to fp32 rounding.
Tolerances: mean within 2e-6 * (|mean| + std), 1/std within 2e-6 relative,
z within 1e-5 * max|z|."""
import zlib

import pytest
import torch

gpu = pytest.mark.gpu

# (name, N, H, W, Cin, Cout, k, s, padding, transpose, bias, math, segments, act)
CASES = [
    # pix2pix G.down2 / D.down2 at the bs16 x 2 pass (generic 128 x 256 bf16x6 tiles)
    ("G.down2", 32, 128, 128, 64, 128, 4, 2, "same", False, False, "bf16x6", 2, "lrelu"),
    # G.up7: Conv2DTranspose forward on the phase-halo kernel (4 sub-pixel phases)
    ("G.up7", 32, 64, 64, 256, 64, 4, 2, "same", True, False, "bf16x6", 2, "relu"),
    # a smaller generic-tile layer with S = 1, and ragged generic tiles (M % 64 != 0) whose
    # 32-row groups meet the segment boundary exactly
    ("G.down3.s1", 8, 64, 64, 128, 256, 4, 2, "same", False, False, "bf16x6", 1, "lrelu"),
    ("gen.ragged", 64, 30, 30, 64, 128, 4, 2, "same", False, True, "bf16x6", 2, "lrelu"),
    # SRGAN residual conv in mixed_float16 (fp16 halo kernel, 24 x 24: ragged patches, bias)
    ("SR.res.fp16", 32, 24, 24, 64, 64, 3, 1, "same", False, True, "fp16", 1, "none"),
    # SR discriminator convs: stride 2 and 64 -> 128 (fp16), 3x3 bf16x6 halo with bias
    ("SR.D.s2.fp16", 16, 96, 96, 64, 64, 3, 2, "same", False, True, "fp16", 2, "lrelu"),
    ("SR.D.128", 64, 48, 48, 64, 128, 3, 1, "same", False, True, "bf16x6", 2, "lrelu"),
    # ragged halo patches on both axes
    ("halo.ragged", 64, 45, 37, 64, 128, 3, 1, "same", False, True, "bf16x6", 2, "lrelu"),
]


def _ref_bn(y, S, gamma, beta, mm, mv, momentum, eps):
    """fp64 Keras BN training statistics per segment (moving stats in segment order)."""
    C = y.shape[-1]
    yd = y.double().reshape(S, -1, C)
    mean = yd.mean(1)
    var = yd.var(1, unbiased=False)
    n = yd.shape[1]
    mm, mv = mm.double().clone(), mv.double().clone()
    for s in range(S):
        mm -= (mm - mean[s]) * (1 - momentum)
        mv -= (mv - var[s] * n / (n - 1)) * (1 - momentum)
    return mean, var, mm, mv


@gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_epilogue_bn_stats_match_fp64(case):
    from dgan import ops
    name, N, H, W, Cin, Cout, k, s, pad, tr, has_bias, math_mode, S, act = case
    torch.manual_seed(zlib.crc32(name.encode()))
    dev = torch.device("cuda")
    d = ops.ConvDesc(N, H, W, Cin, Cout, k, s, pad, tr, math=math_mode)
    bns = ops.BnStatsBuf(dev)
    st = bns.for_conv(d, S)
    assert st is not None and st.R == d.bnstats_groups(S) > 0, f"{name}: plan writes no epilogue statistics"
    x = torch.randn(N, H, W, Cin, device=dev)
    w = torch.randn(*d.weight_shape, device=dev) * (1.0 / (k * (Cin ** 0.5)))
    b = torch.randn(Cout, device=dev) * 0.5 if has_bias else None
    y0 = torch.empty(d.out_shape, device=dev)
    y1 = torch.empty(d.out_shape, device=dev)
    d.fwd(x, w, y0, bias=b)
    st.segs.fill_(-7)
    d.fwd(x, w, y1, bias=b, bn_stats=st)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1), f"{name}: the statistics epilogue changed the conv output"
    segs = st.segs.cpu()
    assert int(segs.min()) >= -1 and int(segs.max()) == S - 1, f"{name}: group segments {segs.unique()}"

    gamma = 1.0 + 0.1 * torch.randn(Cout, device=dev)
    beta = 0.1 * torch.randn(Cout, device=dev)
    mm0, mv0 = 0.1 * torch.randn(Cout, device=dev), 1.0 + 0.1 * torch.rand(Cout, device=dev)
    outs = []
    for use in (st, None):
        mean = torch.empty(S, Cout, device=dev)
        inv = torch.empty(S, Cout, device=dev)
        mm, mv = mm0.clone(), mv0.clone()
        z = torch.empty_like(y1)
        ops.bn_fwd_train(y1, gamma, beta, mean, inv, mm, mv, z, act=act, alpha=0.3, momentum=0.99, eps=1e-3,
                         segments=S, stats=use)
        outs.append((mean, inv, mm, mv, z))
    torch.cuda.synchronize()
    rmean, rvar, rmm, rmv = _ref_bn(y1.cpu(), S, gamma.cpu(), beta.cpu(), mm0.cpu(), mv0.cpu(), 0.99, 1e-3)
    rinv = 1.0 / torch.sqrt(rvar + 1e-3)
    mean, inv, mm, mv, z = [t.double().cpu() for t in outs[0]]
    scale = rmean.abs() + rvar.sqrt()
    assert ((mean - rmean).abs() <= 2e-6 * scale + 1e-12).all(), f"{name}: mean {(mean - rmean).abs().max():.3e}"
    assert ((inv - rinv).abs() <= 2e-6 * rinv).all(), f"{name}: invstd rel {((inv - rinv) / rinv).abs().max():.3e}"
    assert torch.allclose(mm, rmm, rtol=1e-5, atol=1e-6) and torch.allclose(mv, rmv, rtol=1e-5, atol=1e-6)
    # z from the epilogue statistics vs the statistics pass (same apply kernel)
    z_pass = outs[1][4].double().cpu()
    assert (z - z_pass).abs().max() <= 1e-5 * z_pass.abs().max(), f"{name}: z differs from the statistics pass"
    # and vs fp64 act(BN(y))
    C = Cout
    yd = y1.double().cpu().reshape(S, -1, C)
    zr = (yd - rmean[:, None]) * rinv[:, None] * gamma.double().cpu() + beta.double().cpu()
    if act == "lrelu":
        zr = torch.where(zr > 0, zr, 0.3 * zr)
    elif act == "relu":
        zr = zr.clamp_min(0)
    zr = zr.reshape(z.shape)
    assert (z - zr).abs().max() <= 1e-5 * zr.abs().max(), f"{name}: z vs fp64 {(z - zr).abs().max():.3e}"


@gpu
def test_epilogue_bn_stats_refused_where_plan_cannot():
    """Split-K plans (the deep U-Net layers) report no groups and refuse the call."""
    from dgan import ops
    dev = torch.device("cuda")
    d = ops.ConvDesc(32, 4, 4, 512, 512, 4, 2, "same")
    assert d.bnstats_groups(2) == 0
    x = torch.randn(32, 4, 4, 512, device=dev)
    w = torch.randn(*d.weight_shape, device=dev)
    y = torch.empty(d.out_shape, device=dev)
    st = ops.BnStats(torch.empty(3 * 512 * 8, device=dev), torch.empty(8, dtype=torch.int32, device=dev), 8, 2)
    with pytest.raises(ops.DGError):
        d.fwd(x, w, y, bn_stats=st)
