"""CPU oracle for the pix2pix training step — TEST INFRASTRUCTURE ONLY.

A float64 NumPy restatement of the reference's hot path, written from the
reference sources and from the documented TensorFlow semantics it relies on.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker; the product path (dgan/, libdgan.so)
never imports it.

PARITY STATUS: parity unpinned against TensorFlow itself.  The reference
(pmcbride/denoise-gan) ships no tests, fixtures or golden vectors, TensorFlow
is not installable in this container, and the trained .h5 weights are
absent.  This oracle is pinned instead by (1) hand-worked
known-answer tests of each TF semantic it restates (tests/test_oracle.py),
and (2) an independent torch fp64 autograd restatement of the same graph
(oracle/torch_p2p.py) whose gradients must agree with the hand-written
backward below to ~1e-10.

What it restates (file:line in /root/reference):
  architecture   pix2pix.py:105-226   (downsample :110-123, upsample :125-142,
                                        Generator :144-192, Discriminator :194-220)
  losses         pix2pix.py:74-103
  step order     train_pix2pix.py:33-71 (both tapes from one forward, Adam G then D)
  value range    dataloader.py:161-177 (inputs in [-1, 1])
TF/Keras semantics (each checked by a known-answer test):
  1 'same' padding: total = max((ceil(H/s)-1)*s + k - H, 0), before = total//2
  2 Conv2DTranspose 'same' = adjoint of that conv, output H*s
  3 LeakyReLU alpha 0.3; grad `features > 0 ? g : alpha*g`; ReLU grad 0 at 0
  4 BN eps 1e-3, biased batch variance; moving stats momentum 0.99 with the
    Bessel-corrected variance (TF FusedBatchNormV3)
  5 BCE-with-logits max(z,0) - z*y + log1p(exp(-|z|)), mean over all logits
  6 tf.image.total_variation per image: sum |dh| + sum |dw| over all channels
  7 MSE/MAE: mean over all elements; d|x|/dx at 0 is 0
  8 Keras Adam = TF ApplyAdam: alpha = lr*sqrt(1-b2^t)/(1-b1^t),
    m += (g-m)(1-b1), v += (g^2-v)(1-b2), p -= m*alpha/(sqrt(v)+eps)
  9 initialisers: kernels N(0, 0.02), BN gamma 1 beta 0, biases 0
Dropout: Keras' RNG stream cannot be reproduced; both this oracle and the
HIP path use the counter-based hash `dropout_keep` below (bit-identical).
The VGG19 content loss needs ImageNet weights that are unavailable offline;
train_step takes the VGG19 weights to use (PV; None = the term is 0) and
evaluates the term through oracle/sr_oracle.py's VGG19 restatement.
"""
import numpy as np

# ---------------------------------------------------------------------------
# configuration / parameter layout (shared vocabulary with dgan.nets)
# ---------------------------------------------------------------------------
ALPHA = 0.3          # Keras LeakyReLU default (pix2pix.py:121, :213)
BN_EPS = 1e-3        # Keras BatchNormalization default
BN_MOMENTUM = 0.99
LOSS_WEIGHTS = dict(gan=1e-3, l1=1.0, l2=1.0, tv=1e-5, identity=1.0, content=1.0)  # pix2pix.py:75-92


def g_layer_specs(width=1, out_ch=3):
    """Generator layers (pix2pix.py:147-173). width divides every filter count."""
    f = lambda c: max(1, c // width)
    downs = [("down1", 3, f(64), False), ("down2", f(64), f(128), True), ("down3", f(128), f(256), True),
             ("down4", f(256), f(512), True), ("down5", f(512), f(512), True), ("down6", f(512), f(512), True),
             ("down7", f(512), f(512), True), ("down8", f(512), f(512), True)]
    ups = []
    cin = f(512)
    up_f = [512, 512, 512, 512, 256, 128, 64]
    for u in range(7):
        cout = f(up_f[u])
        skip_c = downs[6 - u][2]
        ups.append((f"up{u + 1}", cin, cout, u < 3))
        cin = cout + skip_c
    last = ("last", cin, out_ch)
    return downs, ups, last


def d_layer_specs(width=1):
    """Discriminator layers (pix2pix.py:200-218)."""
    f = lambda c: max(1, c // width)
    return [("down1", 6, f(64), False), ("down2", f(64), f(128), True), ("down3", f(128), f(256), True),
            ("conv", f(256), f(512), True), ("last", f(512), 1, False)]


def g_variables(width=1):
    """(name, shape) of the generator's trainable variables, Keras order."""
    downs, ups, last = g_layer_specs(width)
    out = []
    for name, ci, co, bn in downs:
        out.append((f"{name}/kernel", (4, 4, ci, co)))
        if bn:
            out += [(f"{name}/gamma", (co,)), (f"{name}/beta", (co,))]
    for name, ci, co, _ in ups:
        out += [(f"{name}/kernel", (4, 4, co, ci)), (f"{name}/gamma", (co,)), (f"{name}/beta", (co,))]
    out += [("last/kernel", (4, 4, last[2], last[1])), ("last/bias", (last[2],))]
    return out


def d_variables(width=1):
    out = []
    for name, ci, co, bn in d_layer_specs(width):
        out.append((f"{name}/kernel", (4, 4, ci, co)))
        if bn:
            out += [(f"{name}/gamma", (co,)), (f"{name}/beta", (co,))]
    out.append(("last/bias", (1,)))
    return out


def init_variables(var_list, seed):
    """Seeded Keras-style init: kernels N(0, 0.02) (pix2pix.py:111), gamma 1, beta/bias 0.
    Draw order = variable order, numpy PCG64; float32 like the Keras variables."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, shape in var_list:
        if name.endswith("/kernel"):
            out[name] = (rng.standard_normal(shape) * 0.02).astype(np.float32)
        elif name.endswith("/gamma"):
            out[name] = np.ones(shape, np.float32)
        else:
            out[name] = np.zeros(shape, np.float32)
    return out


def bn_state_names(var_list):
    return [n.rsplit("/", 1)[0] for n, _ in var_list if n.endswith("/gamma")]


def init_bn_states(var_list):
    st = {}
    for layer in bn_state_names(var_list):
        c = None
        for n, s in var_list:
            if n == f"{layer}/gamma":
                c = s[0]
        st[f"{layer}/moving_mean"] = np.zeros(c, np.float32)
        st[f"{layer}/moving_variance"] = np.ones(c, np.float32)
    return st


def synthetic_pair(batch, size, seed=0):
    """Seeded noisy/clean pair: clean y = tanh(2 * bilinear-up(N(0,1) at 1/8 res)),
    noisy x = clip(y + N(0, 0.1^2), -1, 1); both NHWC float32 in [-1, 1] (dataloader.py:173-175)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    lo = max(1, size // 8)
    z = rng.standard_normal((batch, lo + 1, lo + 1, 3))
    # bilinear upsample (align-corners style) to size x size
    t = np.linspace(0.0, lo, size)
    i0 = np.minimum(np.floor(t).astype(int), lo - 1)
    fr = t - i0
    zr = z[:, i0, :, :] * (1 - fr)[None, :, None, None] + z[:, i0 + 1, :, :] * fr[None, :, None, None]
    zc = zr[:, :, i0, :] * (1 - fr)[None, None, :, None] + zr[:, :, i0 + 1, :] * fr[None, None, :, None]
    y = np.tanh(2.0 * zc)
    x = np.clip(y + 0.1 * rng.standard_normal(y.shape), -1.0, 1.0)
    return np.ascontiguousarray(x, dtype=np.float32), np.ascontiguousarray(y, dtype=np.float32)


# ---------------------------------------------------------------------------
# dropout hash (bit-identical to csrc/common.h dg::dropout_keep)
# ---------------------------------------------------------------------------
def _mix32(x):
    x = np.asarray(x, dtype=np.uint32)
    x = x ^ (x >> np.uint32(16))
    x = x * np.uint32(0x7FEB352D)
    x = x ^ (x >> np.uint32(15))
    x = x * np.uint32(0x846CA68B)
    x = x ^ (x >> np.uint32(16))
    return x


def dropout_mask(seed, step, n, rate):
    """keep-mask for flat element indices 0..n-1 (Keras Dropout(0.5) stand-in)."""
    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint32)
        s = _mix32(np.uint32(step) * np.uint32(0x9E3779B9) + np.uint32(0x632BE5AB))
        h = _mix32(np.uint32(seed) ^ s ^ _mix32(idx + np.uint32(0x85EBCA6B)))
        u = (h >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return u >= np.float32(rate)


def dropout_seed(base, layer_idx, pass_idx):
    return (base * 1000003 + layer_idx * 7919 + pass_idx * 104729) & 0xFFFFFFFF


# ---------------------------------------------------------------------------
# layer primitives (float64)
# ---------------------------------------------------------------------------
def tf_same_pads(size, k, s):
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


def _windows(xp, kh, kw, sh, sw, Ho, Wo):
    N, Hp, Wp, C = xp.shape
    st = xp.strides
    return np.lib.stride_tricks.as_strided(
        xp, shape=(N, Ho, Wo, kh, kw, C), strides=(st[0], st[1] * sh, st[2] * sw, st[1], st[2], st[3]),
        writeable=False)


def conv_fwd(x, w, s, pads):
    """x [N,H,W,Ci], w HWIO -> [N,Ho,Wo,Co]"""
    kh, kw, Ci, Co = w.shape
    pt, pb, pl, pr = pads
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    N, Hp, Wp, _ = xp.shape
    Ho, Wo = (Hp - kh) // s + 1, (Wp - kw) // s + 1
    cols = _windows(xp, kh, kw, s, s, Ho, Wo).reshape(N * Ho * Wo, kh * kw * Ci)
    return (cols @ w.reshape(-1, Co)).reshape(N, Ho, Wo, Co)


def conv_bwd_filter(x, dy, kshape, s, pads):
    kh, kw, Ci, Co = kshape
    pt, pb, pl, pr = pads
    xp = np.pad(x, ((0, 0), (pt, pb), (pl, pr), (0, 0)))
    N, Ho, Wo, _ = dy.shape
    cols = _windows(xp, kh, kw, s, s, Ho, Wo).reshape(N * Ho * Wo, kh * kw * Ci)
    return (cols.T @ dy.reshape(-1, Co)).reshape(kh, kw, Ci, Co)


def conv_bwd_data(dy, w, s, pads, in_hw):
    kh, kw, Ci, Co = w.shape
    N, Ho, Wo, _ = dy.shape
    H, W = in_hw
    pt, pb, pl, pr = pads
    dcols = (dy.reshape(-1, Co) @ w.reshape(-1, Co).T).reshape(N, Ho, Wo, kh, kw, Ci)
    dxp = np.zeros((N, H + pt + pb, W + pl + pr, Ci))
    for i in range(kh):
        for j in range(kw):
            dxp[:, i:i + s * (Ho - 1) + 1:s, j:j + s * (Wo - 1) + 1:s, :] += dcols[:, :, :, i, j, :]
    return dxp[:, pt:pt + H, pl:pl + W, :]


def convT_pads(H, k, s):
    """Conv2DTranspose(padding='same'): output H*s; pads of the equivalent conv."""
    Ho = H * s
    total = max((H - 1) * s + k - Ho, 0)
    return Ho, (total // 2, total - total // 2)


def convT_fwd(x, w, s):
    """Keras Conv2DTranspose 'same': x [N,H,W,Cin], w [k,k,F,Cin] -> [N,H*s,W*s,F]"""
    N, H, W, _ = x.shape
    Ho, (pt, pb) = convT_pads(H, w.shape[0], s)
    Wo, (pl, pr) = convT_pads(W, w.shape[1], s)
    return conv_bwd_data(x, w, s, (pt, pb, pl, pr), (Ho, Wo))


def convT_bwd_data(dy, w, s, in_hw):
    H, W = in_hw
    _, (pt, pb) = convT_pads(H, w.shape[0], s)
    _, (pl, pr) = convT_pads(W, w.shape[1], s)
    return conv_fwd(dy, w, s, (pt, pb, pl, pr))


def convT_bwd_filter(x, dy, kshape, s):
    H, W = x.shape[1:3]
    _, (pt, pb) = convT_pads(H, kshape[0], s)
    _, (pl, pr) = convT_pads(W, kshape[1], s)
    return conv_bwd_filter(dy, x, kshape, s, (pt, pb, pl, pr))


def lrelu(v, a=ALPHA):
    return np.where(v > 0, v, a * v)


def bn_train(y, gamma, beta, eps=BN_EPS):
    C = y.shape[-1]
    yf = y.reshape(-1, C)
    mu = yf.mean(0)
    var = ((yf - mu) ** 2).mean(0)
    inv = 1.0 / np.sqrt(var + eps)
    xh = (y - mu) * inv
    return gamma * xh + beta, dict(mu=mu, var=var, inv=inv, xh=xh, n=yf.shape[0])


def bn_bwd(dbn, c, gamma):
    C = dbn.shape[-1]
    d = dbn.reshape(-1, C)
    xh = c["xh"].reshape(-1, C)
    dbeta = d.sum(0)
    dgamma = (d * xh).sum(0)
    dy = gamma * c["inv"] * (d - d.mean(0) - xh * (d * xh).mean(0))
    return dy.reshape(dbn.shape), dgamma, dbeta


def bn_update_moving(state, prefix, c, momentum=BN_MOMENTUM):
    n = c["n"]
    unb = c["var"] * n / max(n - 1, 1)
    mm = state[f"{prefix}/moving_mean"].astype(np.float64)
    mv = state[f"{prefix}/moving_variance"].astype(np.float64)
    state[f"{prefix}/moving_mean"] = (mm - (mm - c["mu"]) * (1 - momentum)).astype(np.float32)
    state[f"{prefix}/moving_variance"] = (mv - (mv - unb) * (1 - momentum)).astype(np.float32)


# ---------------------------------------------------------------------------
# generator / discriminator
# ---------------------------------------------------------------------------
def _p(params, name):
    return params[name].astype(np.float64)


def generator_forward(params, x, width=1, training=True, states=None, drop_rate=0.5, drop_seed=0, step=0,
                      pass_idx=0):
    """pix2pix.py:144-192.  Returns (output, cache)."""
    downs, ups, last = g_layer_specs(width)
    h = x.astype(np.float64)
    cache = dict(inputs=[], ys=[], bn=[], zs=[], masks=[])
    skips = []
    for li, (name, ci, co, use_bn) in enumerate(downs):
        pads = tf_same_pads(h.shape[1], 4, 2) + tf_same_pads(h.shape[2], 4, 2)
        y = conv_fwd(h, _p(params, f"{name}/kernel"), 2, pads)
        bc = None
        if use_bn:
            if training:
                b, bc = bn_train(y, _p(params, f"{name}/gamma"), _p(params, f"{name}/beta"))
                if states is not None:
                    bn_update_moving(states, name, bc)
            else:
                b = bn_infer(y, params, states, name)
        else:
            b = y
        z = lrelu(b)
        cache["inputs"].append((h, pads)); cache["ys"].append(y); cache["bn"].append((bc, b)); cache["zs"].append(z)
        skips.append(z)
        h = z
    skip_list = list(reversed(skips[:-1]))
    cache["up"] = []
    for u, (name, ci, co, drop) in enumerate(ups):
        hin = h
        y = convT_fwd(hin, _p(params, f"{name}/kernel"), 2)
        if training:
            b, bc = bn_train(y, _p(params, f"{name}/gamma"), _p(params, f"{name}/beta"))
            if states is not None:
                bn_update_moving(states, name, bc)
        else:
            b, bc = bn_infer(y, params, states, name), None
        mask = None
        if training and drop and drop_rate > 0:
            seed = dropout_seed(drop_seed, u, pass_idx)
            mask = dropout_mask(seed, step, b.size, drop_rate).reshape(b.shape)
            d = np.where(mask, b / (1.0 - drop_rate), 0.0)
        else:
            d = b
        z = np.maximum(d, 0.0)
        h = np.concatenate([z, skip_list[u]], axis=-1)
        cache["up"].append(dict(hin=hin, y=y, bc=bc, d=d, mask=mask, cz=co))
    pre = convT_fwd(h, _p(params, "last/kernel"), 2) + _p(params, "last/bias")
    out = np.tanh(pre)
    cache["last_in"] = h
    cache["out"] = out
    return out, cache


def bn_infer(y, params, states, name, eps=BN_EPS):
    mm = states[f"{name}/moving_mean"].astype(np.float64)
    mv = states[f"{name}/moving_variance"].astype(np.float64)
    return (y - mm) / np.sqrt(mv + eps) * _p(params, f"{name}/gamma") + _p(params, f"{name}/beta")


def generator_backward(params, cache, dout, width=1, drop_rate=0.5):
    downs, ups, last = g_layer_specs(width)
    g = {}
    out = cache["out"]
    dpre = dout * (1.0 - out * out)
    g["last/bias"] = dpre.sum(axis=(0, 1, 2))
    g["last/kernel"] = convT_bwd_filter(cache["last_in"], dpre, params["last/kernel"].shape, 2)
    dh = convT_bwd_data(dpre, _p(params, "last/kernel"), 2, cache["last_in"].shape[1:3])
    dskip = [None] * 8
    for u in range(6, -1, -1):
        name, ci, co, drop = ups[u]
        c = cache["up"][u]
        dz = dh[..., :co]
        dskip[6 - u] = dh[..., co:]
        dd = dz * (c["d"] > 0)
        if c["mask"] is not None:
            db = np.where(c["mask"], dd / (1.0 - drop_rate), 0.0)
        else:
            db = dd
        dy, dgam, dbet = bn_bwd(db, c["bc"], _p(params, f"{name}/gamma"))
        g[f"{name}/gamma"], g[f"{name}/beta"] = dgam, dbet
        g[f"{name}/kernel"] = convT_bwd_filter(c["hin"], dy, params[f"{name}/kernel"].shape, 2)
        dh = convT_bwd_data(dy, _p(params, f"{name}/kernel"), 2, c["hin"].shape[1:3])
    for li in range(7, -1, -1):
        name, ci, co, use_bn = downs[li]
        dz = dh if dskip[li] is None else dh + dskip[li]
        bc, b = cache["bn"][li]
        dbn = dz * np.where(b > 0, 1.0, ALPHA)
        if use_bn:
            dy, dgam, dbet = bn_bwd(dbn, bc, _p(params, f"{name}/gamma"))
            g[f"{name}/gamma"], g[f"{name}/beta"] = dgam, dbet
        else:
            dy = dbn
        hin, pads = cache["inputs"][li]
        g[f"{name}/kernel"] = conv_bwd_filter(hin, dy, params[f"{name}/kernel"].shape, 2, pads)
        if li > 0:
            dh = conv_bwd_data(dy, _p(params, f"{name}/kernel"), 2, pads, hin.shape[1:3])
    return g


def discriminator_forward(params, inp, tar, width=1, training=True, states=None):
    """pix2pix.py:194-220 -> logits [N,30,30,1] at 256^2."""
    specs = d_layer_specs(width)
    h = np.concatenate([inp.astype(np.float64), tar.astype(np.float64)], axis=-1)
    cache = []
    for name, ci, co, use_bn in specs:
        if name.startswith("down"):
            s, pads = 2, tf_same_pads(h.shape[1], 4, 2) + tf_same_pads(h.shape[2], 4, 2)
        else:
            s, pads = 1, (1, 1, 1, 1)  # ZeroPadding2D() then 'valid' (pix2pix.py:206-218)
        y = conv_fwd(h, _p(params, f"{name}/kernel"), s, pads)
        if name == "last":
            y = y + _p(params, "last/bias")
            cache.append(dict(name=name, hin=h, s=s, pads=pads))
            return y, cache
        bc = None
        if use_bn:
            if training:
                b, bc = bn_train(y, _p(params, f"{name}/gamma"), _p(params, f"{name}/beta"))
                if states is not None:
                    bn_update_moving(states, name, bc)
            else:
                b = bn_infer(y, params, states, name)
        else:
            b = y
        z = lrelu(b)
        cache.append(dict(name=name, hin=h, s=s, pads=pads, bc=bc, b=b, bn=use_bn))
        h = z
    raise AssertionError("unreachable")


def discriminator_backward(params, cache, dlogits, need_input_grad=False, need_param_grad=True):
    g = {}
    dh = dlogits
    dinput = None
    for li in range(len(cache) - 1, -1, -1):
        c = cache[li]
        name = c["name"]
        if name == "last":
            dy = dh
            if need_param_grad:
                g["last/bias"] = dy.sum(axis=(0, 1, 2))
        else:
            dbn = dh * np.where(c["b"] > 0, 1.0, ALPHA)
            if c["bn"]:
                dy, dgam, dbet = bn_bwd(dbn, c["bc"], _p(params, f"{name}/gamma"))
                if need_param_grad:
                    g[f"{name}/gamma"], g[f"{name}/beta"] = dgam, dbet
            else:
                dy = dbn
        if need_param_grad:
            g[f"{name}/kernel"] = conv_bwd_filter(c["hin"], dy, params[f"{name}/kernel"].shape, c["s"], c["pads"])
        if li > 0 or need_input_grad:
            dh = conv_bwd_data(dy, _p(params, f"{name}/kernel"), c["s"], c["pads"], c["hin"].shape[1:3])
            if li == 0:
                dinput = dh
    return g, dinput


# ---------------------------------------------------------------------------
# losses (pix2pix.py:74-103)
# ---------------------------------------------------------------------------
def bce_logits(z, y):
    return np.maximum(z, 0) - z * y + np.log1p(np.exp(-np.abs(z)))


def sigmoid(z):
    return 1.0 / (1.0 + np.exp(-z))


def losses_and_grads(gen, tgt, ident, zr, zf, w=LOSS_WEIGHTS, content=0.0):
    """Returns (tuple8, grads) with tuple8 in train_step order (train_pix2pix.py:71)."""
    gen = gen.astype(np.float64); tgt = tgt.astype(np.float64)
    d = tgt - gen
    n = d.size
    B = d.shape[0]
    dh = d[:, 1:] - d[:, :-1]
    dw = d[:, :, 1:] - d[:, :, :-1]
    tv = np.abs(dh).sum() + np.abs(dw).sum()
    gtv = np.zeros_like(d)
    gtv[:, 1:] += np.sign(dh); gtv[:, :-1] -= np.sign(dh)
    gtv[:, :, 1:] += np.sign(dw); gtv[:, :, :-1] -= np.sign(dw)
    gan = w["gan"] * bce_logits(zf, 1.0).mean()
    l1 = w["l1"] * np.abs(d).mean()
    l2 = w["l2"] * (d * d).mean()
    var = w["tv"] * tv / B
    cont = w["content"] * content
    if ident is not None:
        di = ident.astype(np.float64) - tgt
        idl = w["identity"] * np.abs(di).mean()
        dident = w["identity"] * np.sign(di) / n
    else:
        idl, dident = 0.0, None
    disc = bce_logits(zr, 1.0).mean() + bce_logits(zf, 0.0).mean()
    total = gan + l2 + cont + var + l1 + idl
    nl = zf.size
    dgen = -(w["l1"] * np.sign(d) / n + w["l2"] * 2 * d / n + w["tv"] / B * gtv)
    grads = dict(dgen=dgen, dident=dident, dzr_d=(sigmoid(zr) - 1) / nl, dzf_d=sigmoid(zf) / nl,
                 dzf_g=w["gan"] * (sigmoid(zf) - 1) / nl)
    return (total, gan, l1, l2, cont, disc, var, idl), grads


# ---------------------------------------------------------------------------
# Keras Adam (TF ApplyAdam)
# ---------------------------------------------------------------------------
def adam_update(p, g, m, v, t, lr=2e-4, b1=0.5, b2=0.999, eps=1e-7):
    """Returns new (p, m, v); t is the 1-based step.  Arithmetic in float64 on float32 state."""
    p = p.astype(np.float64); m = m.astype(np.float64); v = v.astype(np.float64)
    alpha = lr * np.sqrt(1 - b2 ** t) / (1 - b1 ** t)
    m = m + (g - m) * (1 - b1)
    v = v + (g * g - v) * (1 - b2)
    p = p - m * alpha / (np.sqrt(v) + eps)
    return p.astype(np.float32), m.astype(np.float32), v.astype(np.float32)


# ---------------------------------------------------------------------------
# the training step (train_pix2pix.py:33-71)
# ---------------------------------------------------------------------------
class P2PState:
    def __init__(self, width=1, seed=1234, drop_rate=0.5, drop_seed=7, identity=True, loss_weights=None):
        self.width = width
        self.gvars = g_variables(width)
        self.dvars = d_variables(width)
        self.G = init_variables(self.gvars, seed)
        self.D = init_variables(self.dvars, seed + 1)
        self.Gs = init_bn_states(self.gvars)
        self.Ds = init_bn_states(self.dvars)
        self.Gm = {k: np.zeros_like(v) for k, v in self.G.items()}
        self.Gv = {k: np.zeros_like(v) for k, v in self.G.items()}
        self.Dm = {k: np.zeros_like(v) for k, v in self.D.items()}
        self.Dv = {k: np.zeros_like(v) for k, v in self.D.items()}
        self.iterations = 0
        self.drop_rate = drop_rate
        self.drop_seed = drop_seed
        self.identity = identity
        self.w = dict(LOSS_WEIGHTS) if loss_weights is None else dict(loss_weights)


def content_value_and_grad(PV, gen, tgt):
    """VGG19 content loss MSE(vgg(pre(tgt))/12.75, vgg(pre(gen))/12.75) (pix2pix.py:45-51) and its
    gradient w.r.t. gen, float64, through oracle/sr_oracle.py's VGG19 restatement (torch autograd)."""
    import torch
    from . import sr_oracle as S
    PVt = {k: torch.tensor(np.asarray(v, np.float64)) for k, v in PV.items()}
    g = torch.tensor(np.asarray(gen, np.float64), requires_grad=True)
    c = S.content_loss(PVt, torch.tensor(np.asarray(tgt, np.float64)), g)
    dg = torch.autograd.grad(c, g)[0]
    return float(c.detach()), dg.numpy()


def train_step(st, x, y, return_grads=False, apply=True, PV=None):
    """One train_step (train_pix2pix.py:33-71).  PV: VGG19 weights of the content term
    (pix2pix.py:87; None = term 0)."""
    step = st.iterations
    gen, cg = generator_forward(st.G, x, st.width, True, st.Gs, st.drop_rate, st.drop_seed, step, 0)
    ident, ci = (None, None)
    if st.identity:
        ident, ci = generator_forward(st.G, y, st.width, True, st.Gs, st.drop_rate, st.drop_seed, step, 1)
    zr, cdr = discriminator_forward(st.D, x, y, st.width, True, st.Ds)
    zf, cdf = discriminator_forward(st.D, x, gen, st.width, True, st.Ds)
    content, dcont = (0.0, None) if PV is None else content_value_and_grad(PV, gen, y)
    vals, lg = losses_and_grads(gen, y, ident, zr, zf, st.w, content=content)
    gDr, _ = discriminator_backward(st.D, cdr, lg["dzr_d"])
    gDf, _ = discriminator_backward(st.D, cdf, lg["dzf_d"])
    gD = {k: gDr[k] + gDf[k] for k in gDr}
    _, dinp = discriminator_backward(st.D, cdf, lg["dzf_g"], need_input_grad=True, need_param_grad=False)
    dgen = lg["dgen"] + dinp[..., 3:]
    if dcont is not None:
        dgen = dgen + st.w["content"] * dcont
    gG = generator_backward(st.G, cg, dgen, st.width, st.drop_rate)
    if st.identity:
        gGi = generator_backward(st.G, ci, lg["dident"], st.width, st.drop_rate)
        gG = {k: gG[k] + gGi[k] for k in gG}
    if apply:
        t = st.iterations + 1
        for k in st.G:
            st.G[k], st.Gm[k], st.Gv[k] = adam_update(st.G[k], gG[k], st.Gm[k], st.Gv[k], t)
        for k in st.D:
            st.D[k], st.Dm[k], st.Dv[k] = adam_update(st.D[k], gD[k], st.Dm[k], st.Dv[k], t)
        st.iterations += 1
    out = dict(losses=vals, gen=gen, ident=ident, logits_real=zr, logits_fake=zf)
    if return_grads:
        out["gG"] = gG
        out["gD"] = gD
    return out
