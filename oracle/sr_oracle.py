"""CPU oracle for the SRGAN / FastSRGAN / Autoencoder training steps and the
VGG19 content loss — TEST INFRASTRUCTURE ONLY.

A float64 torch-CPU restatement (forward written by hand from the reference
sources, gradients by autograd).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may use it, and only as the checker; the product
path (dgan/, libdgan.so) never imports it.  It does not import dgan either:
the only thing it shares with the product is the variable-naming scheme
("<layer>/<kernel|bias|gamma|beta|alpha|depthwise_kernel>") so a test can
hand both the same weights.

PARITY STATUS: parity unpinned against TensorFlow itself (TensorFlow is not
installable here and the reference ships no fixtures).  The
TF semantics restated below are pinned by known-answer tests in
tests/test_sr_oracle.py; the layer conventions shared with the pix2pix
oracle (padding, BN, BCE, TV, Adam) are the ones oracle/p2p_oracle.py
documents and tests.

What it restates (file:line in /root/reference):
  SRGAN G         srgan.py:129-188   conv-BN(gamma~N(1,.02))-PReLU, 16 x [conv-BN-ReLU-conv-BN + skip],
                                      conv-BN + long skip, scale//2 x [conv3 256 -> depth_to_space 2 -> PReLU],
                                      conv1x1(3) + tanh
  SR D            srgan.py:232-272 = fsrgan.py:216-258 (autoencoder.py:188-229 adds a sigmoid)
  FastSRGAN G     fsrgan.py:99-214   inverted residual blocks (fsrgan.py:112-177)
  Autoencoder G   autoencoder.py:89-185
  VGG19           keras.applications.VGG19 to block5_conv4; preprocess_input caffe mode
  content loss    srgan.py:69-76     MSE(vgg(pre(hr))/12.75, vgg(pre(sr))/12.75)
  steps           train_srgan.py:61-118, train_fsrgan.py:61-120, train_autoencoder.py:66-112
  Adam + ExponentialDecay(lr, 100000, 0.1, staircase), D lr x5 (srgan.py:34-49)
TF semantics (beyond those of p2p_oracle):
  S1 PReLU(shared_axes=[1,2]) = relu(x) - alpha * relu(-x), alpha per channel
  S2 tf.nn.depth_to_space NHWC block b: out[n, h*b+i, w*b+j, c] = in[n, h, w, (i*b+j)*C + c]
  S3 DepthwiseConv2D 3x3 'same' stride 1: per-channel correlation, kernel [3,3,C,1]
  S4 MaxPool2D(2,2): max over 2x2 windows, gradient to the first maximum; UpSampling2D(2) nearest: replication
  S5 vgg19.preprocess_input (caffe): RGB->BGR, minus (103.939, 116.779, 123.68)
  S6 Keras BinaryCrossentropy() on a Sigmoid output in graph mode = BCE with the logits
  S7 ExponentialDecay staircase: lr * rate^floor(iterations / steps), iterations before the update
  S8 mixed_float16 (fp16=1): GEMM operands rounded to fp16 as the HIP path's DG_MATH_FP16 does them
     (FP16 below), gradients through the GEMMs at the optimizer's loss scale; LossScaleOptimizer
     'dynamic' (2^15, x2 after 2000 finite steps, /2 and skip on inf/nan)
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from .decisions import of as _dec

BN_EPS = 1e-3
VGG_MEAN_BGR = (103.939, 116.779, 123.68)


# --------------------------------------------------------------------------
# layers (NHWC tensors, Keras kernel layouts)
# --------------------------------------------------------------------------
def tf_same_pads(size, k, s):
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


def _conv_plain(x, w, s):
    k = w.shape[0]
    xt = x.permute(0, 3, 1, 2)
    pt, pb = tf_same_pads(xt.shape[2], k, s)
    pl, pr = tf_same_pads(xt.shape[3], k, s)
    xt = F.pad(xt, (pl, pr, pt, pb))
    return F.conv2d(xt, w.permute(3, 2, 0, 1), stride=s).permute(0, 2, 3, 1)


# ---- mixed_float16 emulation (S8): the HIP path's DG_MATH_FP16 rounds both
# operands of each eligible conv GEMM to fp16 and accumulates exactly enough
# (fp32); the backward GEMMs see the loss-scaled gradient, rounded to fp16.
# FP16 = None: plain fp64 convs; else {"scale": current loss scale}.
FP16 = None


def _q16(t):
    r = t.to(torch.float16)
    ft = FP16.get("flip_tau") if FP16 is not None else None
    if ft:
        tau, seed = ft if isinstance(ft, tuple) else (ft, 0)
        sel = None
        if seed:
            # (a seeded half of the near-tie elements: one more realisation of the flips an fp32
            # value may take; the n-th rounded operand of the step draws from seed and n)
            FP16["flip_n"] = n = FP16.get("flip_n", 0) + 1
            g = torch.Generator().manual_seed(int(seed) * 1000003 + n)
            sel = torch.rand(t.shape, generator=g, dtype=torch.float64) < 0.5
        r = _flip_near_ties(t, r, tau, sel)
    return r.to(t.dtype)


def _flip_near_ties(t, r, tau, sel=None):
    """Tie sensitivity (test diagnostics only): the elements of t whose fp64 value lies
    within tau fp16 ulps of the midpoint between its two fp16 neighbours -- where an
    fp32 value of the same quantity may round to the other neighbour -- take the OTHER
    neighbour (only where sel, a boolean mask of t's shape, is set, when given).  r: t
    rounded to fp16 (RNE)."""
    mag = r.abs().view(torch.int16).to(torch.int32)      # fp16 magnitude bits
    up = t.abs() > r.abs().to(t.dtype)                   # the other neighbour is further from 0
    other_mag = torch.where(up, mag + 1, torch.clamp(mag - 1, min=0))
    other = other_mag.to(torch.int16).view(torch.float16).to(t.dtype) * torch.where(t < 0, -1.0, 1.0).to(t.dtype)
    rd = r.to(t.dtype)
    mid = (rd + other) / 2
    near = (t - mid).abs() < tau * (rd - other).abs()
    near &= torch.isfinite(other) & (other_mag != mag)
    if sel is not None:
        near &= sel
    return torch.where(near, other.to(torch.float16), r)


def fp16_ops(ci, co):
    """Which GEMMs of a conv run in fp16 on the HIP path (include/dgan.h DG_MATH_FP16):
    (fwd, input grad, weight grad)."""
    return (ci % 32 == 0 and co % 16 == 0, ci >= 8 and co % 32 == 0, ci % 16 == 0 and co % 16 == 0)


class _F16Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, s):
        q = fp16_ops(w.shape[2], w.shape[3])
        ctx.save_for_backward(x, w)
        ctx.s, ctx.q = s, q
        return _conv_plain(_q16(x), _q16(w), s) if q[0] else _conv_plain(x, w, s)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        sc = FP16["scale"]
        dyq = _q16(dy * sc) / sc
        dx = dw = None
        with torch.enable_grad():
            if ctx.needs_input_grad[0]:
                xx = x.detach().requires_grad_()
                y = _conv_plain(xx, _q16(w) if ctx.q[1] else w, ctx.s)
                dx = torch.autograd.grad(y, xx, dyq if ctx.q[1] else dy)[0]
            if ctx.needs_input_grad[1]:
                ww = w.detach().requires_grad_()
                y = _conv_plain(_q16(x) if ctx.q[2] else x, ww, ctx.s)
                dw = torch.autograd.grad(y, ww, dyq if ctx.q[2] else dy)[0]
        return dx, dw, None


def conv(x, w, b=None, s=1):
    """Conv2D 'same': x NHWC, w HWIO (fp16-operand GEMMs while FP16 is set)."""
    y = _F16Conv.apply(x, w, s) if FP16 is not None else _conv_plain(x, w, s)
    return y if b is None else y + b


def dwconv3(x, k, b=None):
    """S3: DepthwiseConv2D(3, 'same', stride 1); k [3,3,C,1]."""
    C = x.shape[-1]
    xt = F.pad(x.permute(0, 3, 1, 2), (1, 1, 1, 1))
    wt = k[..., 0].permute(2, 0, 1).unsqueeze(1)  # [C,1,3,3]
    y = F.conv2d(xt, wt, bias=b, groups=C)
    return y.permute(0, 2, 3, 1)


class BNStats:
    """Moving statistics, updated like TF's fused BN (unbiased variance)."""

    def __init__(self):
        self.mean, self.var = {}, {}


def bn(x, gamma, beta, name, stats, momentum=0.99, eps=BN_EPS, training=True):
    if not training:
        m = torch.as_tensor(stats.mean[name])
        v = torch.as_tensor(stats.var[name])
        return (x - m) / torch.sqrt(v + eps) * gamma + beta
    mu = x.mean(dim=(0, 1, 2))
    var = ((x - mu) ** 2).mean(dim=(0, 1, 2))
    n = x.shape[0] * x.shape[1] * x.shape[2]
    C = x.shape[-1]
    m0 = stats.mean.get(name, np.zeros(C))
    v0 = stats.var.get(name, np.ones(C))
    mu_d = mu.detach().numpy()
    var_u = var.detach().numpy() * n / max(n - 1, 1)
    stats.mean[name] = m0 * momentum + mu_d * (1 - momentum)
    stats.var[name] = v0 * momentum + var_u * (1 - momentum)
    return (x - mu) / torch.sqrt(var + eps) * gamma + beta


def prelu(x, alpha):
    """S1."""
    a = alpha.reshape(-1)
    return F.relu(x) - a * F.relu(-x)


def depth_to_space(x, b):
    """S2."""
    N, H, W, CB = x.shape
    C = CB // (b * b)
    y = x.reshape(N, H, W, b, b, C).permute(0, 1, 3, 2, 4, 5)
    return y.reshape(N, H * b, W * b, C)


def maxpool2(x):
    """S4: the gradient goes to ONE element per window, the first maximum in
    row-major window order (TF MaxPoolGrad routes to the forward argmax;
    torch's amax would split it between tied elements)."""
    N, H, W, C = x.shape
    x = x[:, :H // 2 * 2, :W // 2 * 2]
    win = x.reshape(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(N, H // 2, W // 2, C, 4)
    idx = win.detach().argmax(dim=-1, keepdim=True)  # first occurrence of the max
    return win.gather(-1, idx)[..., 0]


def upsample2(x):
    return x.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2)


def lrelu(x, a):
    return torch.where(x > 0, x, a * x)


# --------------------------------------------------------------------------
# networks
# --------------------------------------------------------------------------
def srgan_generator(P, x, stats, scale=4, n_blocks=16, training=True, dec=None):
    """srgan.py:129-188.  dec: oracle.decisions.Decisions (activation sites by layer name)."""
    dec = _dec(dec)
    n = conv(x, P["conv2d/kernel"])
    n = bn(n, P["batch_normalization/gamma"], P["batch_normalization/beta"], "batch_normalization", stats,
           training=training)
    n = dec.prelu("p_re_lu", n, P["p_re_lu/alpha"])
    temp = n
    for i in range(n_blocks):
        nn_ = conv(n, P[f"block_{i}_conv1/kernel"])
        nn_ = dec.relu(f"block_{i}_bn1", bn(nn_, P[f"block_{i}_bn1/gamma"], P[f"block_{i}_bn1/beta"],
                                            f"block_{i}_bn1", stats, training=training))
        nn_ = conv(nn_, P[f"block_{i}_conv2/kernel"])
        nn_ = bn(nn_, P[f"block_{i}_bn2/gamma"], P[f"block_{i}_bn2/beta"], f"block_{i}_bn2", stats,
                 training=training)
        n = n + nn_
    n = conv(n, P["conv2d_post/kernel"])
    n = bn(n, P["batch_normalization_post/gamma"], P["batch_normalization_post/beta"], "batch_normalization_post",
           stats, training=training)
    n = n + temp
    for i in range(scale // 2):
        n = conv(n, P[f"deconv_{i}_conv/kernel"], P[f"deconv_{i}_conv/bias"])
        n = dec.prelu(f"deconv_{i}_p_re_lu", depth_to_space(n, 2), P[f"deconv_{i}_p_re_lu/alpha"])
    return torch.tanh(conv(n, P["conv2d_out/kernel"], P["conv2d_out/bias"]))


def sr_discriminator(P, x, stats, df=32, training=True, dec=None):
    """srgan.py:232-272 (logits)."""
    dec = _dec(dec)
    spec = [(df, 1, False), (df, 2, True), (df, 1, True), (df, 2, True),
            (df * 2, 1, True), (df * 2, 2, True), (df * 2, 1, True), (df * 2, 2, True)]
    h = x
    for i, (f, s, use_bn) in enumerate(spec):
        h = conv(h, P[f"d{i + 1}_conv/kernel"], P[f"d{i + 1}_conv/bias"], s)
        if use_bn:
            h = bn(h, P[f"d{i + 1}_bn/gamma"], P[f"d{i + 1}_bn/beta"], f"d{i + 1}_bn", stats, momentum=0.8,
                   training=training)
        h = dec.lrelu(f"d{i + 1}_bn" if use_bn else f"d{i + 1}_conv", h, 0.2)
    return conv(h, P["logits/kernel"], P["logits/bias"])


def fsrgan_generator(P, x, stats, gf=32, n_blocks=6, training=True, dec=None):
    """fsrgan.py:99-214."""
    dec = _dec(dec)

    def B(h, name, momentum=0.99):
        return bn(h, P[f"{name}/gamma"], P[f"{name}/beta"], name, stats, momentum=momentum, training=training)

    c1 = dec.prelu("p_re_lu", B(conv(x, P["conv2d/kernel"], P["conv2d/bias"]), "batch_normalization"),
                   P["p_re_lu/alpha"])
    r = c1
    for bid in range(n_blocks):
        inp = r
        h = r
        if bid:
            pre = f"block_{bid}_"
            h = conv(h, P[pre + "expand/kernel"], P[pre + "expand/bias"])
            h = dec.relu(pre + "expand_BN", B(h, pre + "expand_BN", 0.999))
        else:
            pre = "expanded_conv_"
        h = dwconv3(h, P[pre + "depthwise/depthwise_kernel"], P[pre + "depthwise/bias"])
        h = dec.relu(pre + "depthwise_BN", B(h, pre + "depthwise_BN", 0.999))
        h = conv(h, P[pre + "project/kernel"], P[pre + "project/bias"])
        h = B(h, pre + "project_BN", 0.999)
        r = inp + h if inp.shape[-1] == h.shape[-1] else h
    c2 = B(conv(r, P["conv2d_post/kernel"], P["conv2d_post/bias"]), "batch_normalization_post") + c1
    u = c2
    for i in range(2):
        u = conv(u, P[f"deconv_{i}_conv/kernel"], P[f"deconv_{i}_conv/bias"])
        u = dec.prelu(f"deconv_{i}_p_re_lu", depth_to_space(u, 2), P[f"deconv_{i}_p_re_lu/alpha"])
    return torch.tanh(conv(u, P["conv2d_out/kernel"], P["conv2d_out/bias"]))


def autoencoder_generator(P, x, dec=None):
    """autoencoder.py:89-185."""
    dec = _dec(dec)

    def c(h, name, relu=True):
        y = conv(h, P[f"{name}/kernel"], P[f"{name}/bias"])
        return dec.relu(name, y) if relu else torch.tanh(y)

    h = c(c(x, "conv1"), "conv1b")
    pool1 = dec.maxpool2("pool1", h)
    pool2 = dec.maxpool2("pool2", c(pool1, "conv2"))
    pool3 = dec.maxpool2("pool3", c(pool2, "conv3"))
    pool4 = dec.maxpool2("pool4", c(pool3, "conv4"))
    pool5 = dec.maxpool2("pool5", c(pool4, "conv5"))
    h = pool5
    for k, (lvl, skip) in enumerate(zip((6, 7, 8, 9), (pool4, pool3, pool2, pool1))):
        h = torch.cat([dec.relu(f"unpool{4 - k}", upsample2(h)), skip], dim=3)
        h = c(c(h, f"conv{lvl}"), f"conv{lvl}b")
    h = torch.cat([dec.relu("unpool0", upsample2(h)), x], dim=3)
    h = c(c(h, "conv10"), "conv10b")
    return c(h, "conv11", relu=False)


VGG19_BLOCKS = [(64, 2), (128, 2), (256, 4), (512, 4), (512, 4)]


def vgg19(P, x, dec=None):
    """VGG19 to block5_conv4 (post-ReLU); x already preprocessed."""
    dec = _dec(dec)
    h = x
    for b, (_, n) in enumerate(VGG19_BLOCKS):
        for i in range(n):
            name = f"block{b + 1}_conv{i + 1}"
            h = dec.relu(name, conv(h, P[f"{name}/kernel"], P[f"{name}/bias"]))
        if b < 4:
            h = dec.maxpool2(f"block{b + 1}_pool", h)
    return h


def vgg_preprocess(img):
    """S5 applied to ((img + 1) * 255) / 2 (srgan.py:71-72)."""
    x = ((img + 1.0) * 255.0) / 2.0
    x = x.flip(-1)
    return x - torch.tensor(VGG_MEAN_BGR, dtype=x.dtype)


def content_loss(PV, hr, sr, dec_sr=None, dec_hr=None):
    """srgan.py:69-76."""
    fs = vgg19(PV, vgg_preprocess(sr), dec_sr) / 12.75
    fh = vgg19(PV, vgg_preprocess(hr), dec_hr) / 12.75
    return ((fh - fs) ** 2).mean()


# --------------------------------------------------------------------------
# losses and steps
# --------------------------------------------------------------------------
def bce_logits(z, y):
    return (torch.clamp(z, min=0) - z * y + torch.log1p(torch.exp(-z.abs()))).mean()


def total_variation(img):
    """tf.image.total_variation: per image sum |dh| + |dw|."""
    dh = (img[:, 1:] - img[:, :-1]).abs().sum(dim=(1, 2, 3))
    dw = (img[:, :, 1:] - img[:, :, :-1]).abs().sum(dim=(1, 2, 3))
    return dh + dw


def exp_decay(lr, it, steps=100000, rate=0.1, staircase=True):
    """S7."""
    e = it / steps
    return lr * rate ** (math.floor(e) if staircase else e)


def adam_update(p, g, m, v, t, lr, b1=0.9, b2=0.999, eps=1e-7):
    """TF ApplyAdam (see p2p_oracle item 8); t = iterations + 1."""
    lr_t = lr * math.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    m = m + (g - m) * (1 - b1)
    v = v + (g * g - v) * (1 - b2)
    p = p - m * lr_t / (np.sqrt(v) + eps)
    return p, m, v


class SRState:
    """Oracle-side copy of one SR model: weights (float64), BN stats, Adam slots."""

    def __init__(self, kind, PG, PD, PV=None, scale=4, lr=1e-3, n_blocks=16, dtype=np.float64, fp16=False):
        """dtype float32: the fp32 CPU restatement timed by bench.py's cpu_baseline leg.
        fp16: the mixed_float16 emulation (S8) with a dynamic loss scale per optimizer."""
        self.kind = kind
        self.fp16 = fp16
        self.ls = {"G": [2.0 ** 15, 0], "D": [2.0 ** 15, 0]}   # [scale, good steps]
        self.dtype = dtype
        self.PG = {k: np.asarray(v, dtype) for k, v in PG.items()}
        self.PD = {k: np.asarray(v, dtype) for k, v in PD.items()}
        self.PV = None if PV is None else {k: np.asarray(v, dtype) for k, v in PV.items()}
        self.scale, self.lr, self.n_blocks = scale, lr, n_blocks
        self.Gs, self.Ds = BNStats(), BNStats()
        self.mG = {k: np.zeros_like(v) for k, v in self.PG.items()}
        self.vG = {k: np.zeros_like(v) for k, v in self.PG.items()}
        self.mD = {k: np.zeros_like(v) for k, v in self.PD.items()}
        self.vD = {k: np.zeros_like(v) for k, v in self.PD.items()}
        self.iterations = 0

    def generator(self, P, x, training=True, dec=None):
        if self.kind == "srgan":
            return srgan_generator(P, x, self.Gs, self.scale, self.n_blocks, training=training, dec=dec)
        if self.kind == "fsrgan":
            return fsrgan_generator(P, x, self.Gs, training=training, dec=dec)
        return autoencoder_generator(P, x, dec=dec)


def train_step(st, x, y, apply=True, dec=None, flip_tau=None):
    """One step of train_srgan.py:61-118 / train_fsrgan.py:61-120 /
    train_autoencoder.py:66-112 (all three share the gen-loss composition
    content + adv + 0*mse + mae; FSRGAN halves the disc loss).
    Returns dict(losses=(gen_total, adv, mae, mse, content, disc, var),
    gen, gG, gD).  dec: {"G", "Dr", "Df", "Vsr", "Vhr": oracle.decisions.Decisions}
    (any subset) -- the activation decisions of G(x), D(y), D(G(x)) and VGG19
    on G(x) and on y (mask-conditioned parity).  flip_tau (fp16 only, test diagnostics):
    every GEMM operand within flip_tau fp16 ulps of a rounding tie takes the other fp16
    neighbour (_flip_near_ties) -- the tie sensitivity of the mixed_float16 step; a
    (tau, seed) pair with seed > 0 flips a seeded half of those operands instead."""
    global FP16
    dec = dec or {}
    FP16 = {"scale": st.ls["G"][0], "flip_tau": flip_tau} if st.fp16 else None
    try:
        return _train_step(st, x, y, apply, dec)
    finally:
        FP16 = None


def _train_step(st, x, y, apply, dec):
    global FP16
    PG = {k: torch.tensor(v, requires_grad=True) for k, v in st.PG.items()}
    PD = {k: torch.tensor(v, requires_grad=True) for k, v in st.PD.items()}
    PV = None if st.PV is None else {k: torch.tensor(v) for k, v in st.PV.items()}
    xt = torch.tensor(np.asarray(x, st.dtype))
    yt = torch.tensor(np.asarray(y, st.dtype))
    gen = st.generator(PG, xt, dec=dec.get("G"))
    zr = sr_discriminator(PD, yt, st.Ds, dec=dec.get("Dr"))
    zf = sr_discriminator(PD, gen, st.Ds, dec=dec.get("Df"))
    cont = (content_loss(PV, yt, gen, dec.get("Vsr"), dec.get("Vhr")) if PV is not None
            else torch.zeros((), dtype=xt.dtype))
    adv = 1e-3 * bce_logits(zf, 1.0)
    mse = ((yt - gen) ** 2).mean()
    mae = (yt - gen).abs().mean()
    var = 1e-5 * total_variation(yt - gen).mean()
    gen_loss = cont + adv + 0 * mse + mae
    disc = bce_logits(zr, 1.0) + bce_logits(zf, 0.0)
    if st.kind == "fsrgan":
        disc = 0.5 * disc
    # one backward pass for d gen_loss / d G(x) and the G gradients (at G's loss scale)
    gs = torch.autograd.grad(gen_loss, [gen] + list(PG.values()), retain_graph=True)
    dgen, gG = gs[0], gs[1:]
    if st.fp16:
        FP16 = {**FP16, "scale": st.ls["D"][0]}
    gD = torch.autograd.grad(disc, list(PD.values()))
    gG = {k: g.numpy() for k, g in zip(PG, gG)}
    gD = {k: g.numpy() for k, g in zip(PD, gD)}
    finite = {"G": all(np.isfinite(g).all() for g in gG.values()),
              "D": all(np.isfinite(g).all() for g in gD.values())}
    out = dict(losses=tuple(float(v.detach()) for v in (gen_loss, adv, mae, mse, cont, disc, var)),
               gen=gen.detach().numpy(), dgen=dgen.numpy(), gG=gG, gD=gD)
    if apply:
        t = st.iterations + 1
        lrg = exp_decay(st.lr, st.iterations)
        lrd = exp_decay(st.lr * 5, st.iterations)
        if not st.fp16 or finite["G"]:
            for k in st.PG:
                st.PG[k], st.mG[k], st.vG[k] = adam_update(st.PG[k], gG[k], st.mG[k], st.vG[k], t, lrg)
        if not st.fp16 or finite["D"]:
            for k in st.PD:
                st.PD[k], st.mD[k], st.vD[k] = adam_update(st.PD[k], gD[k], st.mD[k], st.vD[k], t, lrd)
        st.iterations += 1
        if st.fp16:   # DynamicLossScale.update (after the apply decision)
            for n in ("G", "D"):
                sc, good = st.ls[n]
                if finite[n]:
                    good += 1
                    if good >= 2000:
                        sc, good = sc * 2, 0
                else:
                    sc, good = max(sc / 2, 1.0), 0
                st.ls[n] = [sc, good]
    return out
