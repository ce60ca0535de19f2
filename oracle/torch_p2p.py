"""Independent restatement of the pix2pix step with torch CPU autograd —
TEST INFRASTRUCTURE ONLY (checker and CPU baseline; never the product path).

Two uses:
  * float64: cross-checks the hand-written backward of oracle/p2p_oracle.py
    (gradients come from autograd here, so a transcription error in either
    restatement shows up as a mismatch);
  * float32, all host cores: the `cpu_baseline` leg of bench.py ("CPU
    restatement of the reference graph"; TensorFlow is not installable here).

Follows pix2pix.py:105-226 (architecture), :74-103 (losses) and
train_pix2pix.py:33-71 (step), with the TF semantics listed in
oracle/p2p_oracle.py.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import p2p_oracle as O
from .decisions import of as _dec


def _pad_same(x, k, s):
    pt, pb = O.tf_same_pads(x.shape[2], k, s)
    pl, pr = O.tf_same_pads(x.shape[3], k, s)
    return F.pad(x, (pl, pr, pt, pb))


def _conv(x, w_hwio, s, pad):
    """NCHW activations, HWIO kernel; pad = 'same' or explicit (t,b,l,r)."""
    k = w_hwio.shape[0]
    xp = _pad_same(x, k, s) if pad == "same" else F.pad(x, (pad[2], pad[3], pad[0], pad[1]))
    return F.conv2d(xp, w_hwio.permute(3, 2, 0, 1).contiguous(), stride=s)


def _convT(x, w_kkfc, s):
    """Keras Conv2DTranspose 'same' (output H*s)."""
    H, W = x.shape[2:]
    Ho, (pt, _) = O.convT_pads(H, w_kkfc.shape[0], s)
    Wo, (pl, _) = O.convT_pads(W, w_kkfc.shape[1], s)
    y = F.conv_transpose2d(x, w_kkfc.permute(3, 2, 0, 1).contiguous(), stride=s)
    return y[:, :, pt:pt + Ho, pl:pl + Wo]


def _bn(y, gamma, beta, eps=O.BN_EPS):
    mu = y.mean(dim=(0, 2, 3), keepdim=True)
    var = ((y - mu) ** 2).mean(dim=(0, 2, 3), keepdim=True)
    return (y - mu) / torch.sqrt(var + eps) * gamma.view(1, -1, 1, 1) + beta.view(1, -1, 1, 1)


def generator(P, x, width, drop_rate=0.5, drop_seed=0, step=0, pass_idx=0, dec=None):
    """dec: oracle.decisions.Decisions on NHWC masks, sites named like the layers."""
    dec = _dec(dec)
    downs, ups, last = O.g_layer_specs(width)
    h = x
    skips = []
    for name, ci, co, bn in downs:
        y = _conv(h, P[f"{name}/kernel"], 2, "same")
        if bn:
            y = _bn(y, P[f"{name}/gamma"], P[f"{name}/beta"])
        h = _nchw(dec.lrelu(name, _nhwc(y), O.ALPHA))
        skips.append(h)
    skips = list(reversed(skips[:-1]))
    for u, (name, ci, co, drop) in enumerate(ups):
        y = _bn(_convT(h, P[f"{name}/kernel"], 2), P[f"{name}/gamma"], P[f"{name}/beta"])
        if drop and drop_rate > 0:
            seed = O.dropout_seed(drop_seed, u, pass_idx)
            # masks are defined on the NHWC element order
            n, c, hh, ww = y.shape
            m = O.dropout_mask(seed, step, y.numel(), drop_rate).reshape(n, hh, ww, c)
            m = torch.from_numpy(m).permute(0, 3, 1, 2).to(y.dtype)
            y = y * m / (1.0 - drop_rate)
        h = torch.cat([_nchw(dec.relu(name, _nhwc(y))), skips[u]], dim=1)
    return torch.tanh(_convT(h, P["last/kernel"], 2) + P["last/bias"].view(1, -1, 1, 1))


def discriminator(P, inp, tar, width, dec=None):
    dec = _dec(dec)
    h = torch.cat([inp, tar], dim=1)
    for name, ci, co, bn in O.d_layer_specs(width):
        if name.startswith("down"):
            y = _conv(h, P[f"{name}/kernel"], 2, "same")
        else:
            y = _conv(h, P[f"{name}/kernel"], 1, (1, 1, 1, 1))
        if name == "last":
            return y + P["last/bias"].view(1, -1, 1, 1)
        if bn:
            y = _bn(y, P[f"{name}/gamma"], P[f"{name}/beta"])
        h = _nchw(dec.lrelu(name, _nhwc(y), O.ALPHA))


def _nhwc(t):
    return t.permute(0, 2, 3, 1)


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def _bce(z, y):
    return (torch.clamp(z, min=0) - z * y + torch.log1p(torch.exp(-z.abs()))).mean()


def _content(PV, yt, gen, dec_sr=None, dec_hr=None):
    """VGG19 content loss (pix2pix.py:45-51) on NCHW tensors, via oracle/sr_oracle.py's restatement."""
    from . import sr_oracle as S
    return S.content_loss(PV, yt.permute(0, 2, 3, 1), gen.permute(0, 2, 3, 1), dec_sr, dec_hr)


def step_grads(Gnp, Dnp, x, y, width=1, drop_rate=0.5, drop_seed=0, step=0, identity=True, weights=None,
               dtype=torch.float64, PV=None, dec=None):
    """One train_step's losses and gradients (no optimizer) -> (tuple8, gG, gD) as numpy float64.
    PV: VGG19 weights for the content term (None: the term is 0).
    dec: {"Gx", "Gy", "Dr", "Df", "Vsr", "Vhr": oracle.decisions.Decisions} (any subset):
    the activation decisions of G(x), G(y), D(real), D(fake) and VGG19 on G(x) / y."""
    dec = dec or {}
    w = dict(O.LOSS_WEIGHTS) if weights is None else weights
    G = {k: torch.tensor(v, dtype=dtype, requires_grad=True) for k, v in Gnp.items()}
    D = {k: torch.tensor(v, dtype=dtype, requires_grad=True) for k, v in Dnp.items()}
    xt = torch.tensor(x, dtype=dtype).permute(0, 3, 1, 2)
    yt = torch.tensor(y, dtype=dtype).permute(0, 3, 1, 2)
    gen = generator(G, xt, width, drop_rate, drop_seed, step, 0, dec=dec.get("Gx"))
    zr = discriminator(D, xt, yt, width, dec=dec.get("Dr"))
    zf = discriminator(D, xt, gen, width, dec=dec.get("Df"))
    d = yt - gen
    gan = w["gan"] * _bce(zf, 1.0)
    tv = w["tv"] * ((d[:, :, 1:] - d[:, :, :-1]).abs().sum() + (d[:, :, :, 1:] - d[:, :, :, :-1]).abs().sum()) / d.shape[0]
    l1 = w["l1"] * d.abs().mean()
    l2 = w["l2"] * (d * d).mean()
    if identity:
        idl = w["identity"] * (generator(G, yt, width, drop_rate, drop_seed, step, 1, dec=dec.get("Gy"))
                               - yt).abs().mean()
    else:
        idl = torch.zeros((), dtype=dtype)
    if PV is not None:
        cont = w["content"] * _content({k: torch.tensor(v, dtype=dtype) for k, v in PV.items()}, yt, gen,
                                       dec.get("Vsr"), dec.get("Vhr"))
    else:
        cont = torch.zeros((), dtype=dtype)
    total = gan + l2 + cont + tv + l1 + idl
    disc = _bce(zr, 1.0) + _bce(zf, 0.0)
    gG = torch.autograd.grad(total, list(G.values()), retain_graph=True)
    gD = torch.autograd.grad(disc, list(D.values()))
    vals = tuple(float(v.detach()) for v in (total, gan, l1, l2, cont, disc, tv, idl))
    return (vals, {k: g.double().numpy() for k, g in zip(G, gG)}, {k: g.double().numpy() for k, g in zip(D, gD)},
            gen.detach().permute(0, 2, 3, 1).double().numpy())


def make_fp32_step(Gnp, Dnp, width=1, lr=2e-4, b1=0.5, b2=0.999, eps=1e-7, PV=None):
    """A full fp32 CPU training step (fwd, both backwards, Keras-Adam; VGG19 content loss when PV is
    given) for the CPU baseline timing."""
    PVt = None if PV is None else {k: torch.tensor(v, dtype=torch.float32) for k, v in PV.items()}
    G = {k: torch.tensor(v, dtype=torch.float32, requires_grad=True) for k, v in Gnp.items()}
    D = {k: torch.tensor(v, dtype=torch.float32, requires_grad=True) for k, v in Dnp.items()}
    opt_state = {"t": 0, "m": {}, "v": {}}

    def adam(params, grads):
        t = opt_state["t"]
        alpha = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
        with torch.no_grad():
            for p, g in zip(params, grads):
                m = opt_state["m"].setdefault(id(p), torch.zeros_like(p))
                v = opt_state["v"].setdefault(id(p), torch.zeros_like(p))
                m.add_((g - m) * (1 - b1))
                v.add_((g * g - v) * (1 - b2))
                p.sub_(m * alpha / (v.sqrt() + eps))

    def step(x, y):
        xt = torch.from_numpy(x).permute(0, 3, 1, 2)
        yt = torch.from_numpy(y).permute(0, 3, 1, 2)
        gen = generator(G, xt, width, 0.5, 0, opt_state["t"], 0)
        zr = discriminator(D, xt, yt, width)
        zf = discriminator(D, xt, gen, width)
        d = yt - gen
        total = (1e-3 * _bce(zf, 1.0) + (d * d).mean() + 1e-5 * (
            (d[:, :, 1:] - d[:, :, :-1]).abs().sum() + (d[:, :, :, 1:] - d[:, :, :, :-1]).abs().sum()) / d.shape[0]
                 + d.abs().mean() + (generator(G, yt, width, 0.5, 0, opt_state["t"], 1) - yt).abs().mean())
        if PVt is not None:
            total = total + _content(PVt, yt, gen)
        disc = _bce(zr, 1.0) + _bce(zf, 0.0)
        gG = torch.autograd.grad(total, list(G.values()), retain_graph=True)
        gD = torch.autograd.grad(disc, list(D.values()))
        opt_state["t"] += 1
        adam(list(G.values()), gG)
        adam(list(D.values()), gD)
        return float(total.detach()), float(disc.detach())

    return step
