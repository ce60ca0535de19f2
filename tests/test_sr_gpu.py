"""SR-family layers and training steps on the HIP path vs the CPU oracles.

Layer kernels (csrc/layers.hip) are checked against torch fp64 autograd of
the oracle's restatement of each TF op (oracle/sr_oracle.py S1-S7); the
fused training steps of SRGAN / FastSRGAN / Autoencoder (dgan.sr_trainer)
against oracle.sr_oracle.train_step on the same weights and synthetic
inputs, VGG19 content loss included (seeded stand-in weights).

Tolerances (fp32 vs fp64): layers 1e-5 relative to the output scale; full
steps: the 7 loss values to 2e-5 relative, generator output |dPSNR| < 0.01 dB
and max-abs 1e-4, every G and D gradient to max-abs 1e-4 (BASELINE.json
north_star; 1e-5 relative for gradients above 10, see _grads_close).  Where ReLU / LeakyReLU / max-pool decisions can tie within fp32
rounding (VGG19, the discriminators), the oracle runs mask-conditioned on the
HIP path's decisions, each override audited as a near-tie (oracle/decisions.py).
"""
import math
import zlib

import numpy as np
import pytest
import torch

from oracle import sr_oracle as S


def _vsrc(cl):
    """(plan, slot, rows) of G(x)'s and of the target's VGG19 activations (ContentLoss)."""
    (pg, rg), (pt, rt) = cl.feature_sources()
    return (pg, 0, rg), (pt, 0, rt)

gpu = pytest.mark.gpu
DEV = "cuda"


def _t(a):
    return torch.as_tensor(np.asarray(a, np.float32)).to(DEV)


def _close(got, ref, rtol=1e-5, atol=0.0, what=""):
    got = got.detach().double().cpu().numpy() if torch.is_tensor(got) else np.asarray(got, np.float64)
    ref = ref.detach().double().cpu().numpy() if torch.is_tensor(ref) else np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (what, got.shape, ref.shape)
    err = np.abs(got - ref).max() if got.size else 0.0
    scale = np.abs(ref).max() if ref.size else 0.0
    assert err <= atol + rtol * scale, f"{what}: max abs err {err:.3e} vs scale {scale:.3e}"
    return err


def _padded(shape, C_ld=None):
    """NHWC device buffer whose pixel stride exceeds C (exercises ld handling)."""
    N, H, W, C = shape
    ld = C_ld or C + 4
    return torch.zeros((N, H, W, ld), device=DEV)[..., :C]


# -------------------------------------------------------------------------
# layers
# -------------------------------------------------------------------------
@gpu
@pytest.mark.parametrize("block,N,H,W,C", [(1, 2, 5, 7, 12), (2, 2, 5, 7, 12), (2, 3, 13, 9, 64), (2, 2, 5, 7, 3),
                                           (1, 2, 6, 5, 3)])
def test_prelu_depth_to_space(block, N, H, W, C):
    """float4 kernels (C % 4 == 0: k_prelu_fwd4 / k_prelu_bwd4, SRGAN's 64-channel shape with
    ragged row chunks) and the one-channel kernels (C = 3)."""
    from dgan import ops
    rng = np.random.default_rng(block * 100 + C)
    y = rng.standard_normal((N, H, W, C * block * block))
    y[0, 0, 0, :3] = 0.0  # exact zeros: gradient 0 (relu' at 0)
    a = rng.standard_normal((1, 1, C)) * 0.3
    dz = rng.standard_normal((N, H * block, W * block, C))
    yt = torch.tensor(y, requires_grad=True)
    at = torch.tensor(a, requires_grad=True)
    zt = S.prelu(S.depth_to_space(yt, block) if block > 1 else yt, at)
    zt.backward(torch.tensor(dz))
    yd, ad, dzd = _t(y), _t(a), _t(dz)
    z = _padded((N, H * block, W * block, C))
    ops.prelu_fwd(yd, ad, z, block=block)
    dy = _padded(yd.shape)
    da = torch.zeros_like(ad)
    ops.prelu_bwd(yd, ad, dzd, dy, dalpha=da, block=block)
    torch.cuda.synchronize()
    _close(z, zt, 1e-6, what="prelu fwd")
    _close(dy, yt.grad, 1e-6, what="prelu dy")
    _close(da, at.grad, 1e-5, what="prelu dalpha")


@gpu
def test_depthwise_conv_fwd_bwd():
    from dgan import ops
    rng = np.random.default_rng(7)
    N, H, W, C = 2, 9, 11, 70
    x = rng.standard_normal((N, H, W, C))
    k = rng.standard_normal((3, 3, C, 1)) * 0.3
    b = rng.standard_normal(C)
    dy = rng.standard_normal((N, H, W, C))
    xt, kt, bt = (torch.tensor(v, requires_grad=True) for v in (x, k, b))
    yt = S.dwconv3(xt, kt, bt)
    yt.backward(torch.tensor(dy))
    xd, kd, bd, dyd = _t(x), _t(k), _t(b), _t(dy)
    y = _padded((N, H, W, C))
    ops.dwconv3_fwd(xd, kd, y, bias=bd)
    dx = _padded((N, H, W, C))
    dx.fill_(1.0)
    ops.dwconv3_bwd_data(dyd, kd, dx, beta=1.0)   # accumulate onto ones
    dk = torch.zeros_like(kd)
    db = torch.zeros_like(bd)
    ops.dwconv3_bwd_filter(xd, dyd, dk, dbias=db)
    torch.cuda.synchronize()
    _close(y, yt, 1e-6, what="dw fwd")
    _close(dx, xt.grad + 1.0, 1e-6, what="dw dx")
    _close(dk, kt.grad, 2e-6, what="dw dk")
    _close(db, bt.grad, 2e-6, what="dw db")


@gpu
def test_maxpool_upsample_fwd_bwd():
    from dgan import ops
    rng = np.random.default_rng(3)
    N, H, W, C = 2, 8, 6, 9
    x = rng.standard_normal((N, H, W, C))
    xt = torch.tensor(x, requires_grad=True)
    pt = S.maxpool2(xt)
    dp = rng.standard_normal(pt.shape)
    pt.backward(torch.tensor(dp))
    xd = _t(x)
    p = _padded(tuple(pt.shape))
    ops.maxpool2_fwd(xd, p)
    dx = _padded((N, H, W, C))
    ops.maxpool2_bwd(xd, _t(dp), dx)
    # upsample + relu
    ut_in = torch.tensor(x, requires_grad=True)
    ut = torch.relu(S.upsample2(ut_in))
    du = rng.standard_normal(ut.shape)
    ut.backward(torch.tensor(du))
    u = _padded(tuple(ut.shape))
    ops.upsample2_relu_fwd(xd, u)
    dxu = _padded((N, H, W, C))
    ops.upsample2_relu_bwd(xd, _t(du), dxu)
    torch.cuda.synchronize()
    _close(p, pt, 1e-7, what="maxpool fwd")   # fp32 rounding of the inputs only
    _close(dx, xt.grad, 1e-7, what="maxpool bwd")
    _close(u, ut, 1e-7, what="upsample fwd")
    _close(dxu, ut_in.grad, 1e-6, what="upsample bwd")


@gpu
def test_vgg_preprocess_and_content_mse():
    from dgan import ops
    rng = np.random.default_rng(5)
    img = rng.uniform(-1, 1, (2, 4, 5, 3))
    it = torch.tensor(img, requires_grad=True)
    zt = S.vgg_preprocess(it)
    dz = rng.standard_normal(zt.shape)
    zt.backward(torch.tensor(dz))
    z = _padded((2, 4, 5, 3))
    ops.vgg_preprocess_fwd(_t(img), z)
    dimg = torch.ones((2, 4, 5, 3), device=DEV)
    ops.vgg_preprocess_bwd(_t(dz), dimg, beta=1.0)
    a = rng.standard_normal((3, 2, 2, 40)) * 50
    b = rng.standard_normal((3, 2, 2, 40)) * 50
    at = torch.tensor(a, requires_grad=True)
    mt = (((torch.tensor(b) - at) / 12.75) ** 2).mean()
    mt.backward()
    out = torch.zeros(1, device=DEV)
    da = torch.zeros((3, 2, 2, 40), device=DEV)
    ops.mse(_t(a), _t(b), out, scale=1 / 12.75, da=da, grad_weight=1.0)
    torch.cuda.synchronize()
    _close(z, zt, 1e-6, what="preprocess fwd")
    _close(dimg, it.grad + 1.0, 1e-6, what="preprocess bwd")
    _close(out[0], mt, 1e-6, what="mse value")
    _close(da, at.grad, 1e-6, what="mse grad")


@gpu
def test_gan_loss_set_matches_oracle():
    from dgan import ops
    rng = np.random.default_rng(11)
    B, H, W = 3, 12, 10
    g = np.tanh(rng.standard_normal((B, H, W, 3)))
    y = np.tanh(rng.standard_normal((B, H, W, 3)))
    zr = rng.standard_normal((B, 2, 2, 1)) * 3
    zf = rng.standard_normal((B, 2, 2, 1)) * 3
    for coef in [(1e-3, 1e-5, 1.0, 1.0, 0.0, 1.0, 0.0), (1e-3, 1e-5, 0.5, 0.7, 0.3, 1.0, 2.0)]:
        gt = torch.tensor(g, requires_grad=True)
        zrt = torch.tensor(zr, requires_grad=True)
        zft = torch.tensor(zf, requires_grad=True)
        yt = torch.tensor(y)
        cont = torch.tensor(0.25, dtype=torch.float64)
        adv = coef[0] * S.bce_logits(zft, 1.0)
        mae = (yt - gt).abs().mean()
        mse = ((yt - gt) ** 2).mean()
        var = coef[1] * S.total_variation(yt - gt).mean()
        total = adv + coef[3] * mae + coef[4] * mse + coef[5] * cont + coef[6] * var
        disc = coef[2] * (S.bce_logits(zrt, 1.0) + S.bce_logits(zft, 0.0))
        dgen_img = torch.autograd.grad(total - adv, gt, retain_graph=True)[0]
        dzf_g = torch.autograd.grad(adv, zft, retain_graph=True)[0]
        dzr_d, dzf_d = torch.autograd.grad(disc, [zrt, zft])
        out = torch.zeros(7, device=DEV)
        dgen = torch.zeros((B, H, W, 3), device=DEV)
        d1, d2, d3 = (torch.zeros((B, 2, 2, 1), device=DEV) for _ in range(3))
        ops.gan_loss(_t(g), _t(y), _t(zr), _t(zf), out, coef, content=_t([0.25]), dgen=dgen, dlogit_real_d=d1,
                     dlogit_fake_d=d2, dlogit_fake_g=d3)
        torch.cuda.synchronize()
        want = [total, adv, mae, mse, cont, disc, var]
        for i, w in enumerate(want):
            _close(out[i], w, 2e-6, atol=1e-9, what=f"loss[{i}]")
        _close(dgen, dgen_img, 1e-5, what="dgen")
        _close(d1, dzr_d, 1e-6, what="dzr_d")
        _close(d2, dzf_d, 1e-6, what="dzf_d")
        _close(d3, dzf_g, 1e-6, what="dzf_g")


@gpu
def test_adam_exponential_decay():
    from dgan import ops
    rng = np.random.default_rng(2)
    n = 1001
    p, g = rng.standard_normal(n), rng.standard_normal(n) * 1e-3
    m, v = rng.standard_normal(n) * 1e-4, rng.uniform(0, 1e-6, n)
    for it in (0, 99999, 100000, 250001):
        dp, dg, dm, dv = _t(p), _t(g), _t(m), _t(v)
        itd = torch.tensor([it], dtype=torch.int32, device=DEV)
        ops.adam_sched(dp, dg, dm, dv, 1e-3, 100000, 0.1, True, 0.9, 0.999, 1e-7, itd)
        rp, rm, rv = S.adam_update(p, g, m, v, it + 1, S.exp_decay(1e-3, it))
        torch.cuda.synchronize()
        _close(dp, rp, 1e-6, what=f"adam p it={it}")
        # step size must reflect the decayed lr
        step = np.abs(dp.cpu().numpy() - p.astype(np.float32)).max()
        assert step <= S.exp_decay(1e-3, it) * 1.01 * math.sqrt(1 - 0.999 ** (it + 1)) / (1 - 0.9 ** (it + 1)) * 4


# layer geometries of the SR family that the pix2pix conv tests do not cover
SR_CONVS = [
    # (name, N, H, W, Cin, Cout, k, s, bias, ld_in)
    ("srgan.res", 2, 12, 12, 64, 64, 3, 1, False, None),
    ("srgan.deconv", 2, 12, 12, 64, 256, 3, 1, True, None),
    ("srgan.out1x1", 2, 24, 24, 64, 3, 1, 1, True, None),
    ("fsrgan.expand", 2, 16, 16, 32, 192, 1, 1, True, None),
    ("fsrgan.project", 2, 16, 16, 192, 32, 1, 1, True, None),
    ("fsrgan.out3x3", 2, 32, 32, 32, 3, 3, 1, True, None),
    ("d.s2", 2, 24, 24, 32, 32, 3, 2, True, None),
    ("d.in3", 2, 24, 24, 3, 32, 3, 1, True, None),
    ("d.logits", 2, 6, 6, 64, 1, 1, 1, True, None),
    ("ae.conv2", 2, 16, 16, 32, 44, 3, 1, True, None),
    ("ae.conv6", 2, 4, 4, 176, 152, 3, 1, True, None),
    ("ae.conv8", 2, 8, 8, 156, 84, 3, 1, True, None),
    ("ae.conv10", 2, 32, 32, 67, 64, 3, 1, True, 68),
    ("ae.slice_in", 2, 8, 8, 76, 100, 3, 1, True, 176),
    ("vgg.c11", 2, 16, 16, 3, 64, 3, 1, True, None),
    ("vgg48.b1", 2, 48, 48, 64, 64, 3, 1, True, None),
    ("vgg48.b2", 2, 24, 24, 128, 128, 3, 1, True, None),
    ("vgg48.b3", 2, 12, 12, 256, 256, 3, 1, True, None),
    ("vgg48.b4", 2, 6, 6, 512, 512, 3, 1, True, None),
    ("vgg48.b5", 2, 3, 3, 512, 512, 3, 1, True, None),
    ("vgg48.b4in", 2, 6, 6, 256, 512, 3, 1, True, None),
    ("vgg48.c11", 2, 48, 48, 3, 64, 3, 1, True, None),
    ("odd.5x5", 2, 5, 5, 64, 64, 3, 1, True, None),
    ("ae.d2", 4, 64, 64, 32, 32, 3, 2, True, None),
    ("ae.d4", 4, 32, 32, 32, 32, 3, 2, True, None),
    ("ae.d5", 4, 16, 16, 32, 64, 3, 1, True, None),
    ("ae.d6", 4, 16, 16, 64, 64, 3, 2, True, None),
    ("odd.7x3", 3, 7, 3, 128, 64, 3, 1, True, None),
    # thread-per-pixel narrow forward (k_narrow_fwd_px, Co 1 / 3, Ci % 4 == 0) at the sizes
    # FastSRGAN's 512x512 output conv runs it (M >= 65536), a ragged M and ldx > Ci
    ("px.fsrgan_out", 1, 512, 512, 32, 3, 3, 1, True, None),
    ("px.co1.ragged", 1, 257, 263, 32, 1, 3, 1, True, 36),
    ("px.co3.1x1.ld", 2, 200, 171, 64, 3, 1, 1, True, 68),
    ("px.co3.small", 3, 9, 13, 32, 3, 3, 1, True, 40),
    # 32-wide GEMM tiles (the SR discriminators' 32-channel layers): fp32 128x32 in all three
    # ops, bf16x6 128x32 input gradient (RC images of 32 columns), fp32 256x32 forward
    ("tile32.s1", 2, 128, 128, 32, 32, 3, 1, True, None),
    ("tile32.s2", 4, 128, 128, 32, 32, 3, 2, True, None),
    ("tile32.fwd256", 8, 256, 256, 32, 32, 3, 2, True, None),
    # 3-channel input conv (SR discriminators' d1): filter gradient on the row-segment kernel
    ("ntile.in3", 2, 128, 128, 3, 32, 3, 1, True, None),
    ("ntile.in3.ragged", 3, 37, 101, 3, 48, 3, 1, True, None),
]


@gpu
@pytest.mark.parametrize("case", SR_CONVS, ids=[c[0] for c in SR_CONVS])
def test_sr_conv_geometries(case):
    from torch_ref import conv2d_ref
    from dgan.ops import ConvDesc
    name, N, H, W, Ci, Co, k, s, bias, ld_in = case
    torch.manual_seed(zlib.crc32(name.encode()))
    d = ConvDesc(N, H, W, Ci, Co, k, s, "same")
    x = torch.randn(N, H, W, Ci, dtype=torch.float64)
    w = torch.randn(*d.weight_shape, dtype=torch.float64) * 0.05
    b = torch.randn(Co, dtype=torch.float64) if bias else None
    dy = torch.randn(N, d.Ho, d.Wo, Co, dtype=torch.float64)
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    br = b.clone().requires_grad_() if bias else None
    yr = conv2d_ref(xr, wr, s, d.pads, br)
    yr.backward(dy)
    xg = _padded((N, H, W, Ci), ld_in or -(-Ci // 4) * 4)
    xg.copy_(x.float())
    wg = w.float().to(DEV)
    bg = b.float().to(DEV) if bias else None
    y = _padded((N, d.Ho, d.Wo, Co), -(-Co // 4) * 4)
    d.fwd(xg, wg, y, bias=bg)
    dx = _padded((N, H, W, Ci), ld_in or -(-Ci // 4) * 4)
    d.bwd_data(dy.float().to(DEV), wg, dx)
    dw = torch.zeros_like(wg)
    db = torch.zeros(Co, device=DEV) if bias else None
    d.bwd_filter(xg, dy.float().to(DEV), dw, dbias=db)
    # masked input gradient: dx * lrelu'(z) for a z = LeakyReLU(.2) output
    z = torch.randn(N, H, W, Ci, dtype=torch.float64)
    zg = _padded((N, H, W, Ci), ld_in or -(-Ci // 4) * 4)
    zg.copy_(z.float())
    dxm = _padded((N, H, W, Ci), ld_in or -(-Ci // 4) * 4)
    d.bwd_data_masked(dy.float().to(DEV), wg, dxm, zg, "lrelu", 0.2)
    torch.cuda.synchronize()
    K = k * k * max(Ci, Co)
    tol = 1e-5 * max(1.0, math.sqrt(K / 1024))
    _close(dxm, xr.grad * torch.where(z > 0, 1.0, 0.2), tol, what="bwd_data_masked")
    _close(y, yr, tol, what="fwd")
    _close(dx, xr.grad, tol, what="bwd_data")
    _close(dw, wr.grad, tol * 4, what="bwd_filter")
    if bias:
        _close(db, br.grad, 1e-5, what="dbias")


# -------------------------------------------------------------------------
# full training steps
# -------------------------------------------------------------------------
class Args:
    def __init__(self, **kw):
        self.crop_size = 32
        self.scale = 4
        self.fp16 = 0
        self.lr = 1e-3
        self.retrain = 0
        self.seed = 21
        self.__dict__.update(kw)


def psnr(img, ref):
    a = (np.asarray(img, np.float64) + 1) / 2
    b = (np.asarray(ref, np.float64) + 1) / 2
    return 10 * math.log10(1.0 / np.mean((a - b) ** 2))


def _grads_close(arena, ref, label, rtol=1e-5, atol=1e-4):
    """max-abs 1e-4 (north star), or 1e-5 of the variable's largest gradient where that is above 10:
    e.g. SRGAN bs32's conv2d_out/bias gradient (max 51, a sum over 3e5 pixels) carries ~3e-6
    relative fp32 accumulation error."""
    worst = 0.0
    for name, g_ref in ref.items():
        g = arena.grad_of(name).detach().double().cpu().numpy()
        err = float(np.abs(g - g_ref).max())
        tol = atol + rtol * float(np.abs(g_ref).max())
        assert err <= tol, f"{label} {name}: max-abs grad diff {err:.3e} > {tol:.3e} (ref max {np.abs(g_ref).max():.3e})"
        worst = max(worst, err)
    return worst


def _synthetic(N, H, W, scale, seed, gray=False):
    from dataloader import synthetic_pair
    x, y = synthetic_pair(N, H, seed=seed)
    if gray:
        x = np.repeat(x.mean(-1, keepdims=True), 3, -1).astype(np.float32)
        y = np.repeat(y.mean(-1, keepdims=True), 3, -1).astype(np.float32)
    if scale > 1:
        x = np.ascontiguousarray(x[:, ::scale, ::scale, :])
    return x, y


def _sr_decisions(tr):
    """The HIP step's activation decisions (G, D real, D fake, VGG19 on G(x) and y) for
    S.train_step(dec=...)."""
    from gpu_decisions import graph_decisions, to_oracle
    dec = {"G": graph_decisions(tr.Gp, 0), "Dr": graph_decisions(tr.Dp, 0), "Df": graph_decisions(tr.Dp, 1)}
    if tr.content is not None:
        N = tr.N
        dec["Vsr"] = graph_decisions(*_vsrc(tr.content)[0])
        dec["Vhr"] = graph_decisions(*_vsrc(tr.content)[1])
    return {k: to_oracle(v) for k, v in dec.items()}


TIE_TOL = 1e-5   # an overridden decision must sit within 1e-5 of its layer's scale of the tie


def _run_step_parity(model_cls, kind, N, H, scale, steps=1, conditioned=False, gray=False, **kw):
    """HIP step vs S.train_step on the same weights and inputs.  conditioned:
    the oracle takes the HIP path's ReLU / LeakyReLU / PReLU / max-pool
    decisions (oracle/decisions.py), audited to be near-ties, so gradients
    compare elementwise even where fp32 and fp64 land on opposite sides of a
    tie (VGG19's 16 ReLUs and 4 pools, the discriminators' LeakyReLUs)."""
    m = model_cls(Args(crop_size=H, scale=scale, **kw))
    st = S.SRState(kind, m.generator.arena.export(), m.discriminator.arena.export(),
                   m.vgg.arena.export() if m.vgg is not None else None, scale=scale, lr=1e-3)
    res = None
    for it in range(steps):
        x, y = _synthetic(N, H, H, scale, seed=50 + it, gray=gray)
        last = it == steps - 1
        tr = m.trainer(x.shape, y.shape)
        loss = tr.step(torch.from_numpy(x).to(DEV), torch.from_numpy(y).to(DEV), apply=not last)
        torch.cuda.synchronize()
        dec = _sr_decisions(tr) if (conditioned and last and steps == 1) else None
        ref = S.train_step(st, x, y, apply=True, dec=dec)
        got = loss.cpu().double().numpy()
        want = np.array(ref["losses"])
        rt = 2e-5 if it == 0 else 5e-4
        assert np.allclose(got, want, rtol=rt, atol=1e-8), (it, got, want)
        res = (m, tr, ref, x, y, dec)
    m, tr, ref, x, y, dec = res
    gen = tr.gen_output.detach().cpu().numpy()
    out = {}
    if steps == 1:
        assert abs(psnr(gen, y) - psnr(ref["gen"], y)) < 0.01
        assert np.abs(gen - ref["gen"]).max() < 1e-4
        if dec is not None:
            from gpu_decisions import audit_ok
            out["overridden"] = audit_ok(dec, TIE_TOL, kind)
        out["G"] = _grads_close(m.generator.arena, ref["gG"], "G")
        out["D"] = _grads_close(m.discriminator.arena, ref["gD"], "D")
        print(f"{kind} parity: worst |dg| G {out['G']:.2e} D {out['D']:.2e}; overridden decisions "
              f"{out.get('overridden', 0)}")
    return m, st


@gpu
def test_srgan_step_parity():
    from srgan import SRGAN
    m, st = _run_step_parity(SRGAN, "srgan", N=2, H=32, scale=4)
    # BN moving statistics after G(x), D(y), D(G(x))
    bn_g = m.generator.bn.export()
    for k, v in st.Gs.mean.items():
        assert np.allclose(bn_g[f"{k}/moving_mean"], v, rtol=1e-4, atol=1e-5), k
    bn_d = m.discriminator.bn.export()
    for k, v in st.Ds.var.items():
        assert np.allclose(bn_d[f"{k}/moving_variance"], v, rtol=1e-4, atol=1e-5), k


@gpu
def test_fsrgan_step_parity_no_content():
    from fsrgan import FastSRGAN
    _run_step_parity(FastSRGAN, "fsrgan", N=2, H=64, scale=4, content_loss=0)


@gpu
def test_fsrgan_step_parity_with_vgg_content():
    from fsrgan import FastSRGAN
    _run_step_parity(FastSRGAN, "fsrgan", N=2, H=64, scale=4, conditioned=True)


@gpu
def test_autoencoder_step_parity_no_content():
    """BASELINE config a: 64x64 grayscale replicated to 3 channels, batch 4.
    On this seed the discriminator's LeakyReLU inputs come within 8.6e-8
    (d1, real pass), 2.5e-7 (d1, fake pass) and 4e-7 (d3) of zero relative
    to their layer's scale (fp64 oracle), i.e. inside fp32 rounding, and one
    slope flip in the 4x4 patch layers moves every upstream D gradient by
    ~1%: the oracle takes the HIP path's decisions (audited near-ties)."""
    from autoencoder import Autoencoder
    _run_step_parity(Autoencoder, "autoencoder", N=4, H=64, scale=1, conditioned=True, content_loss=0)


@gpu
def test_autoencoder_step_parity_with_vgg_content():
    from autoencoder import Autoencoder
    _run_step_parity(Autoencoder, "autoencoder", N=4, H=64, scale=1, conditioned=True)


@gpu
def test_vgg_content_gradient_matches_oracle():
    """VGG19 content loss value and input gradient, elementwise to 1e-5 of the
    scale, with the fp64 oracle taking the HIP path's ReLU / max-pool decisions
    (audited: an overridden decision must be a near-tie within 1e-5 of its
    layer's scale) -- a single flipped near-tie would otherwise move the input
    gradient over its receptive field far beyond 1e-5."""
    from dataloader import synthetic_pair
    from dgan import ops
    from dgan.sr_trainer import ContentLoss, VGGNetwork
    from gpu_decisions import audit_ok, graph_decisions, to_oracle
    vgg = VGGNetwork(seed=11)
    PV = {k: torch.tensor(v.astype(np.float64)) for k, v in vgg.arena.export().items()}
    for N, H in ((2, 32), (2, 64), (4, 32)):
        x, y = synthetic_pair(N, H, seed=3)
        gen = np.tanh(np.arctanh(np.clip(y, -0.99, 0.99)) + 0.3 * np.random.default_rng(0).standard_normal(y.shape))
        gen = gen.astype(np.float32)
        cl = ContentLoss(vgg, N, H, H, torch.device(DEV))
        ws = ops.Workspace()
        ws.get(cl.ws_bytes)
        dg = torch.zeros((N, H, H, 3), device=DEV)
        v = cl.forward(torch.from_numpy(gen).to(DEV), torch.from_numpy(y).to(DEV), ws=ws)
        cl.backward(dg, beta=0.0, ws=ws)
        torch.cuda.synchronize()
        dec = {"Vsr": to_oracle(graph_decisions(*_vsrc(cl)[0])),
               "Vhr": to_oracle(graph_decisions(*_vsrc(cl)[1]))}
        gt = torch.tensor(gen.astype(np.float64), requires_grad=True)
        c = S.content_loss(PV, torch.tensor(y.astype(np.float64)), gt, dec["Vsr"], dec["Vhr"])
        d0 = torch.autograd.grad(c, gt)[0]
        audit_ok(dec, 1e-5, f"content {N}x{H}")
        _close(v[0], c, 2e-6, what=f"content {N}x{H}")
        _close(dg, d0, 1e-5, what=f"content grad {N}x{H}")


@gpu
def test_srgan_full_config_parity():
    """BASELINE configs[2]: SRGAN 4x, 24 -> 96 crops, 16 residual blocks, batch 32, VGG19 content
    loss -- the full-size kernel plans, mask-conditioned, max-abs 1e-4."""
    from srgan import SRGAN
    _run_step_parity(SRGAN, "srgan", N=32, H=96, scale=4, conditioned=True)


@gpu
def test_autoencoder_full_config_parity():
    """BASELINE configs[0]: autoencoder 64x64, batch 4, grayscale replicated to 3 channels, VGG19
    content loss, mask-conditioned, max-abs 1e-4."""
    from autoencoder import Autoencoder
    _run_step_parity(Autoencoder, "autoencoder", N=4, H=64, scale=1, conditioned=True, gray=True)


@gpu
@pytest.mark.timeout(900)
def test_fsrgan_full_size_parity():
    """BASELINE configs[4] at its per-GPU image size: FastSRGAN 128 -> 512, VGG19 content loss at
    512x512, mask-conditioned, max-abs 1e-4.  bs2 (M = 524,288 output pixels) already fires every
    size-dependent plan of the bs8 shard: the narrow output conv, the depthwise kernels at 128x128x192,
    the 512x512 discriminator and VGG19 layers."""
    from fsrgan import FastSRGAN
    _run_step_parity(FastSRGAN, "fsrgan", N=2, H=512, scale=4, conditioned=True)


@gpu
def test_srgan_two_steps_track_oracle():
    """Adam with ExponentialDecay and TTUR (D lr x5): step-2 losses track the oracle."""
    from srgan import SRGAN
    _run_step_parity(SRGAN, "srgan", N=2, H=32, scale=4, steps=2)


@gpu
def test_sr_train_step_tuples():
    import train_autoencoder
    import train_fsrgan
    import train_srgan
    from autoencoder import Autoencoder
    from fsrgan import FastSRGAN
    from srgan import SRGAN
    for mod, cls, H, scale, n in ((train_srgan, SRGAN, 32, 4, 7), (train_fsrgan, FastSRGAN, 32, 4, 8),
                                  (train_autoencoder, Autoencoder, 32, 1, 5)):
        m = cls(Args(crop_size=H, scale=scale, vgg_width=8))
        x, y = _synthetic(2, H, H, scale, seed=1)
        out = mod.train_step(m, x, y)
        assert len(out) == n and all(torch.isfinite(v).item() for v in out)
        g = m.generator(x, training=False)
        assert tuple(g.shape) == (2, H, H, 3)
        d = m.discriminator(y, training=False)
        assert d.shape[-1] == 1
        if cls is Autoencoder:
            assert float(d.min()) >= 0.0 and float(d.max()) <= 1.0  # sigmoid output


@gpu
@pytest.mark.parametrize("kind", ["srgan", "fsrgan"])
def test_sr_step_under_library_wide_f16x3(kind, monkeypatch):
    """DG_CONV_MATH=f16x3 as the library-wide default (include/dgan.h): the SR generators' 64- /
    32-channel convs then get fp16x3 input gradients whose dy comes from a BN / PReLU (no producer
    bound: measured before the conv's backward, dgan/graph.py x3_measure_dy) and fp16x3 x planes
    (measured by the op that splits them) -- the plans build and the step meets the same fp64 bars
    as the default arithmetic (plan construction used to raise)."""
    monkeypatch.setenv("DG_CONV_MATH", "f16x3")
    from dgan import ops
    assert ops.default_conv_math() == ops.MATH_F16X3
    if kind == "srgan":
        from srgan import SRGAN
        _run_step_parity(SRGAN, "srgan", N=2, H=32, scale=4, conditioned=True)
    else:
        from fsrgan import FastSRGAN
        _run_step_parity(FastSRGAN, "fsrgan", N=2, H=64, scale=4, content_loss=0)


@gpu
def test_two_slot_plan_keeps_per_slot_activation_scales(monkeypatch):
    """D(real) and D(fake) are two slots of one GraphPlan sharing its conv
    descriptors.  Under fp16x3 activation planes each slot's kept x planes carry the scale of the
    maxima measured in THAT slot's forward; slot 1's forward must not change the scale slot 0's
    filter gradient reads them back with.  Slot inputs 40x apart (five binades): both forwards then
    both backwards (the SR trainer's order) must give the parameter gradients of two one-slot passes,
    bit for bit."""
    monkeypatch.setenv("DG_CONV_MATH", "f16x3")
    from dgan import ops, zoo
    from dgan.graph import GraphNetwork
    D = GraphNetwork(zoo.sr_discriminator(), seed=5)
    N, H = 2, 32
    two = D.plan(N, H, H, slots=2, train=True)
    one = D.plan(N, H, H, slots=1, train=True)
    assert two.amax is not None and two.amax.shape[0] == 2, "fp16x3 activation planes in play"
    g = torch.Generator().manual_seed(3)
    x0 = (torch.rand(N, H, H, 3, generator=g) * 2 - 1).to(DEV)
    x1 = (40.0 * (torch.rand(N, H, H, 3, generator=g) * 2 - 1)).to(DEV)
    dl0 = (torch.randn(two.out_shape, generator=g) * 1e-2).to(DEV)
    dl1 = (torch.randn(two.out_shape, generator=g) * 1e-2).to(DEV)
    ws = ops.Workspace(DEV)
    ws.get(max(two.ws_bytes, one.ws_bytes))
    two.forward(x0, slot=0, training=True, ws=ws)
    two.forward(x1, slot=1, training=True, ws=ws)
    two.backward(dl0, slot=0, param_beta=0.0, ws=ws)
    two.backward(dl1, slot=1, param_beta=1.0, ws=ws)
    g_two = D.arena.grad.clone()
    one.forward(x0, slot=0, training=True, ws=ws)
    one.backward(dl0, slot=0, param_beta=0.0, ws=ws)
    one.forward(x1, slot=0, training=True, ws=ws)
    one.backward(dl1, slot=0, param_beta=1.0, ws=ws)
    g_one = D.arena.grad.clone()
    torch.cuda.synchronize()
    assert torch.isfinite(g_two).all()
    bad = [n for n, _ in D.arena.var_list
           if not torch.equal(D.arena._v(g_two, n), D.arena._v(g_one, n))]
    assert not bad, f"two-slot gradients differ from the one-slot passes: {bad}"
