"""pix2pix generator / discriminator executors on libdgan.

This replaces what tf.keras + GradientTape do for the reference's
`train_step` (train_pix2pix.py:33-71): instead of a traced autodiff graph,
each network has a static plan — layer descriptors, activation buffers,
and an explicit backward schedule — built once per input shape.

Memory layout (HBM, all fp32 NHWC):
  * trainable variables of a network live in ONE flat arena (plus grad, m,
    v arenas of identical layout), laid out in backward-completion order so
    gradient buckets become final front-to-back (data-parallel all-reduce
    and the single-launch Adam both run over contiguous ranges);
  * the U-Net skip concat (pix2pix.py:188) is zero-copy: each down block
    writes its activation straight into the channel tail of the up block's
    concat buffer, and its gradient is accumulated there in place;
  * the discriminator's input concat (pix2pix.py:200) is a 6-channel buffer
    whose fake half is written directly by the generator's last layer.
"""
import math
import os

import numpy as np
import torch

from . import ops
from .ops import ConvDesc

ALPHA = 0.3       # Keras LeakyReLU default (pix2pix.py:121, :213)
BN_EPS = 1e-3     # Keras BatchNormalization defaults (pix2pix.py:119)
BN_MOMENTUM = 0.99
DROP_RATE = 0.5   # pix2pix.py:138
FEED_DY = not os.environ.get("DG_NO_FEED_DY")  # BN backward writes the conv's dy planes
FEED_X = not os.environ.get("DG_NO_FEED_X")    # BN forward writes the next convs' x planes
DY_PLANES_ONLY = not os.environ.get("DG_DY_FP32")  # ... and then skips the fp32 dy (its readers take the planes)
# fp16x3 activation planes scaled from their producers' bounds (ActBounds); DG_NO_ACT_BOUND: the
# round-4 static 2^-4 (same-box A/B only: |x| < 2 then loses bits)
ACT_BOUNDS = not os.environ.get("DG_NO_ACT_BOUND")
# BN backward of the blocks without dropout takes act'(z) from y and the forward's scale / shift
# (dg_bn_bwd_seg_r) instead of reading z; DG_BN_READ_Z: read z (same-box A/B)
BN_RZ = not os.environ.get("DG_BN_READ_Z")
# D's input gradient into a LeakyReLU block without BN masked in the conv epilogue; DG_NO_MASK_DZ:
# a separate act_bwd pass (same-box A/B)
MASK_DZ = not os.environ.get("DG_NO_MASK_DZ")


def _eb(buf):
    """bytes per element of PlaneBuf buf's format (bf16x6 6, fp16x3 4)"""
    return 4 if buf.fmt == ops.PLANES_F16X3 else 6


def xrows(buf, row0, rows, C):
    """The bytes of PlaneBuf `buf` holding rows [row0, row0 + rows) of a
    [rows, C]-channel tensor's planes (bf16x6 or fp16x3, buf.fmt)."""
    e = _eb(buf)
    return buf.buf[row0 * e * C:(row0 + rows) * e * C]


def plane_rows(buf, t, row0):
    """The bytes of PlaneBuf `buf` holding rows [row0, row0 + rows of t) of a
    [rows, C] tensor's planes (6 bytes per element bf16x6, 4 fp16x3)."""
    C = t.shape[-1]
    rows = t[..., 0].numel()
    e = _eb(buf)
    return buf.buf[row0 * e * C:(row0 + rows) * e * C]


def zplanes(buf, rows, C, col):
    """(bytes, planes C, column) of a BN forward's plane output into PlaneBuf buf: a
    negative planes C names fp16x3 planes (dg_bn_fwd_train_seg_h)."""
    return xrows(buf, 0, rows, C), (-C if buf.fmt == ops.PLANES_F16X3 else C), col


# conv arithmetic of the pix2pix G / D GEMMs (include/dgan.h DG_MATH_*): fp16x3 -- three
# fp16 piece products of pre-scaled operands, gradients scaled from their bound -- by
# default; DG_P2P_MATH=bf16x6 for the six-piece bf16 form
P2P_MATH = os.environ.get("DG_P2P_MATH", "f16x3")


def grad_bounds(descs, planes, device):
    """One dy bound (a max slot) per conv whose dy planes are fp16x3 (written by the BN backward
    producing that dy, dg_bn_bwd_seg_x), set as the conv's dy scale source; None elsewhere
    (the conv measures max |dy| itself where it splits dy)."""
    out = []
    for d, P in zip(descs, planes):
        b = None
        if FEED_DY and P is not None and P.dy is not None and P.dy.fmt == ops.PLANES_F16X3:
            b = ops.max_slot(device=device)
            d.set_grad_scale(dy_m=b)
        out.append(b)
    return out


def x3_planes(P):
    """P keeps fp16x3 x planes (an fp16x3 op of its layer reads x from them)."""
    return P is not None and P.x is not None and P.x.fmt == ops.PLANES_F16X3


class ActBounds:
    """Scale sources of a network's fp16x3 activation planes (include/dgan.h
    dg_conv_set_act_scale): `zb[i]` (a max slot) the bound of BN block i's output written by its
    statistics (dg_bn_fwd_train_seg_x), `in_max` the measured max |input| and `w1[0]` the
    forward weight bound of the first conv (no BN after it: its output planes are scaled from
    in_max x w1).  Each conv whose x planes are fp16x3 reads the source its producer wrote
    them with, so values down to 2^-17 of the tensor's bound keep 22 bits (a static 2^-4
    scale left |x| < 2 -- most of a BN output -- with a subnormal low piece)."""

    def __init__(self, n, device):
        self.zb = ops.max_slot(n, device=device)
        self.in_max = ops.max_slot(device=device)
        self.w1 = torch.zeros(2, dtype=torch.float32, device=device)

    def first_conv(self, x, w):
        """Per forward: max |x| of the network input and the first conv's weight bound."""
        ops.weight_bound(w, self.w1[0:1], zero=self.in_max)   # (zeroes in_max for the absmax)
        ops.absmax(x, self.in_max)

    @property
    def first_src(self):
        return (self.in_max, self.w1[0:1])


# ---------------------------------------------------------------------------
# layer specs (pix2pix.py:147-173, :200-218); `width` divides filter counts
# (tiny variants for tests only; width=1 is the reference model)
# ---------------------------------------------------------------------------
def g_layer_specs(width=1, in_ch=3, out_ch=3):
    f = lambda c: max(1, c // width)
    downs = [("down1", in_ch, f(64), False), ("down2", f(64), f(128), True), ("down3", f(128), f(256), True),
             ("down4", f(256), f(512), True), ("down5", f(512), f(512), True), ("down6", f(512), f(512), True),
             ("down7", f(512), f(512), True), ("down8", f(512), f(512), True)]
    ups = []
    cin = f(512)
    for u, c in enumerate([512, 512, 512, 512, 256, 128, 64]):
        cout = f(c)
        ups.append((f"up{u + 1}", cin, cout, u < 3))
        cin = cout + downs[6 - u][2]
    return downs, ups, ("last", cin, out_ch)


def d_layer_specs(width=1, in_ch=6):
    f = lambda c: max(1, c // width)
    return [("down1", in_ch, f(64), False), ("down2", f(64), f(128), True), ("down3", f(128), f(256), True),
            ("conv", f(256), f(512), True), ("last", f(512), 1, False)]


def g_variables(width=1):
    """(name, shape) in Keras trainable_variables order."""
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


def dropout_seed(base, layer_idx, pass_idx):
    return (base * 1000003 + layer_idx * 7919 + pass_idx * 104729) & 0xFFFFFFFF


def init_variables(var_list, seed):
    """Keras-style init from a seeded numpy PCG64 stream: kernels N(0, 0.02)
    (pix2pix.py:111, :126, :168, :195), BN gamma 1 / beta 0, biases 0."""
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


# ---------------------------------------------------------------------------
# flat parameter arena
# ---------------------------------------------------------------------------
class Arena:
    """Trainable variables (+grad, Adam m/v) of one network in flat device buffers."""
    ALIGN = 64  # floats; keeps every variable 256-byte aligned for vector loads

    def __init__(self, var_list, device, layout_order=None):
        self.var_list = list(var_list)
        self.shapes = dict(var_list)
        order = layout_order or [n for n, _ in var_list]
        assert sorted(order) == sorted(self.shapes)
        self.offsets = {}
        off = 0
        for n in order:
            self.offsets[n] = off
            off += -(-int(np.prod(self.shapes[n])) // self.ALIGN) * self.ALIGN
        self.layout = list(order)
        self.numel = off
        self.device = device
        self.data = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        self.m = torch.zeros(off, dtype=torch.float32, device=device)
        self.v = torch.zeros(off, dtype=torch.float32, device=device)
        self.iterations = torch.zeros(1, dtype=torch.int32, device=device)

    def _v(self, buf, name):
        o = self.offsets[name]
        shape = self.shapes[name]
        return buf[o:o + int(np.prod(shape))].view(shape)

    def param(self, name):
        return self._v(self.data, name)

    def grad_of(self, name):
        return self._v(self.grad, name)

    def end_offset(self, name):
        return self.offsets[name] + int(np.prod(self.shapes[name]))

    def load(self, values):
        for n, a in values.items():
            self.param(n).copy_(torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float32))
        self.version = getattr(self, "version", 0) + 1  # host-side weight writes (frozen nets' plane reuse)

    def export(self, buf=None):
        return {n: self._v(self.data if buf is None else buf, n).detach().cpu().numpy().copy()
                for n, _ in self.var_list}

    @property
    def count(self):
        return sum(int(np.prod(s)) for s in self.shapes.values())


class BNState:
    """Non-trainable moving statistics of every BN layer of a network."""

    def __init__(self, channels, device):
        self.mean = {k: torch.zeros(c, device=device) for k, c in channels.items()}
        self.var = {k: torch.ones(c, device=device) for k, c in channels.items()}

    def export(self):
        out = {}
        for k in self.mean:
            out[f"{k}/moving_mean"] = self.mean[k].cpu().numpy()
            out[f"{k}/moving_variance"] = self.var[k].cpu().numpy()
        return out

    def load(self, values):
        for k in self.mean:
            if f"{k}/moving_mean" in values:
                self.mean[k].copy_(torch.as_tensor(values[f"{k}/moving_mean"]))
                self.var[k].copy_(torch.as_tensor(values[f"{k}/moving_variance"]))


def _bn_channels(var_list):
    return {n.rsplit("/", 1)[0]: s[0] for n, s in var_list if n.endswith("/gamma")}


def _empty(shape, device):
    return torch.empty(shape, dtype=torch.float32, device=device)


# ---------------------------------------------------------------------------
# U-Net generator plan (pix2pix.py:144-192)
# ---------------------------------------------------------------------------
class GeneratorPlan:
    """Static forward/backward schedule of the U-Net for one input shape.

    halves: independent images sets batched into ONE pass (half 0 = G(x),
    half 1 = G(target) for the identity loss, pix2pix.py:90).  The convs run
    once over all halves*N images -- twice the GEMM rows of two separate
    passes, which fills the chip on the deep layers -- while BatchNorm
    (statistics, moving averages, dropout masks) is applied per half, exactly
    as the reference's two separate generator calls."""

    def __init__(self, N, H, W, width, arena, bn_state, device, halves=1, train=True, conv_math=None):
        self.N, self.H, self.W, self.width = N, H, W, width
        math_ = conv_math or P2P_MATH
        self.halves = halves
        NT = N * halves
        self.NT = NT
        self.arena, self.bn = arena, bn_state
        self.device = device
        self.downs, self.ups, self.last = g_layer_specs(width)
        self.train = train
        if H % (1 << 8) or W % (1 << 8):
            # 8 stride-2 blocks need H, W divisible by 2^8 for the skip shapes to line up
            raise ValueError(f"pix2pix generator needs H, W divisible by 256, got {H}x{W}")
        # descriptors over all halves
        self.ddesc, self.udesc = [], []
        h, w = H, W
        self.down_hw = []
        for name, ci, co, _ in self.downs:
            d = ConvDesc(NT, h, w, ci, co, 4, 2, "same", math=math_)
            self.ddesc.append(d)
            h, w = d.Ho, d.Wo
            self.down_hw.append((h, w))
        for name, ci, co, _ in self.ups:
            d = ConvDesc(NT, h, w, ci, co, 4, 2, "same", transpose=True, math=math_)
            self.udesc.append(d)
            h, w = d.Ho, d.Wo
        self.ldesc = ConvDesc(NT, h, w, self.last[1], self.last[2], 4, 2, "same", transpose=True, math=math_)
        for d, (name, *_) in zip(self.ddesc + self.udesc + [self.ldesc], self.downs + self.ups + [self.last]):
            d.label = f"G.{name}"
        self.out_shape = self.ldesc.out_shape
        # activations
        s = {}
        s["cat"] = []
        for u, (name, ci, co, _) in enumerate(self.ups):
            d = self.udesc[u]
            skip_c = self.downs[6 - u][2]
            s["cat"].append(_empty((NT, d.Ho, d.Wo, co + skip_c), device))
        s["z8"] = _empty((NT,) + self.down_hw[7] + (self.downs[7][2],), device)
        s["yd"] = [(_empty((NT,) + self.down_hw[i] + (self.downs[i][2],), device) if self.downs[i][3] else None)
                   for i in range(8)]
        s["yu"] = [_empty(self.udesc[u].out_shape, device) for u in range(7)]
        s["mean"] = {}
        s["inv"] = {}
        for name, _, co, bn in self.downs + [(n, a, b, True) for n, a, b, _ in self.ups]:
            if bn:  # [half, channel]: one segmented BN call covers the halves
                s["mean"][name] = _empty((halves, co), device)
                s["inv"][name] = _empty((halves, co), device)
        s["x"] = None
        s["out"] = None
        self.s = s
        # gradient buffers
        if train:
            self.dcat = [torch.empty_like(c) for c in s["cat"]]
            self.dz8 = torch.empty_like(s["z8"])
            maxdy = max([d.N * d.Ho * d.Wo * d.Cout for d in self.ddesc + self.udesc + [self.ldesc]])
            self.dy = _empty((maxdy,), device)
        # bf16x6 operand planes shared by the ops of each layer (x: fwd ->
        # bwd_filter, w: fwd -> bwd_data, dy: bwd_filter -> bwd_data)
        descs = self.ddesc + self.udesc + [self.ldesc]
        self.planes = ops.plan_planes(descs, device) if train else [None] * len(descs)
        # down1 (conv + LeakyReLU, no BN) writes down2's x planes in its epilogue
        if train and FEED_X and self.planes[1].x is not None:
            self.planes[0].fwd_out = self.planes[1].x
        self.gbound = grad_bounds(descs, self.planes, device) if train else [None] * len(descs)
        # fp16x3 activation planes scaled from their producers' bounds (ActBounds): down l's BN
        # output -> zb[l] (down l+1's x), up u's BN output with the skip half of its concat ->
        # zb[8+u] (up u+1's x), down1's conv output -> (max |x|, down1's weight bound) (down2's x)
        self.ab = None
        if train and ACT_BOUNDS and any(x3_planes(P) for P in self.planes):
            self.ab = ActBounds(16, device)
            for k, d in enumerate(descs):
                if not x3_planes(self.planes[k]):
                    continue
                # (plane index k: 0-7 down1-down8, 8-14 up1-up7, 15 last; the x of k >= 2 is the BN
                # output of block k-1, zb[k-1])
                d.set_act_scale(x=self.ab.first_src if k == 1 else self.ab.zb[k - 1])
            if x3_planes(self.planes[1]) and FEED_X:
                self.ddesc[0].set_act_scale(y=self.ab.first_src)
        self.ws_bytes = max([d.max_ws() for d in self.ddesc + self.udesc + [self.ldesc]] + [self._bn_ws_max()])

    @property
    def slots(self):
        return [self.s]

    def _bn_ws_max(self):
        m = 0
        for d in self.ddesc + self.udesc:
            m = max(m, ops.bn_workspace_bytes(self.N * d.Ho * d.Wo, d.Cout, self.halves))
        return m

    def _half(self, t, h):
        return t[h * self.N:(h + 1) * self.N]

    # views ---------------------------------------------------------------
    def z_view(self, s, l):
        """activation of down block l (post LeakyReLU) inside its concat buffer"""
        if l == 7:
            return s["z8"]
        u = 6 - l
        co = self.ups[u][2]
        return s["cat"][u][..., co:]

    def dz_view(self, l):
        if l == 7:
            return self.dz8
        u = 6 - l
        return self.dcat[u][..., self.ups[u][2]:]

    def _dy(self, d, C):
        return self.dy[: d.N * d.Ho * d.Wo * C].view(d.N, d.Ho, d.Wo, C)

    # forward --------------------------------------------------------------
    def forward(self, x, out, slot=0, training=True, ws=None, drop_rate=DROP_RATE, drop_seed=0, step_dev=None):
        """x [halves*N,H,W,3] view; writes the tanh output into `out` (any NHWC view of that batch)."""
        s = self.s
        s["x"], s["out"] = x, out
        A = self.arena
        P = self._fwd_planes()
        feed = FEED_X and training

        def xplanes(k):  # plane index k's kept x planes (None: its ops split x themselves)
            return P[k].x if feed and P[k] is not None else None

        ab = self.ab
        if ab is not None:
            # down2's x planes: (max |x|, down1's bound) -- also in a training plan's inference pass,
            # whose down1 still writes them
            ab.first_conv(x, A.param("down1/kernel"))
        h = x
        for l, (name, ci, co, bn) in enumerate(self.downs):
            d = self.ddesc[l]
            z = self.z_view(s, l)
            if not bn:
                d.fwd(h, A.param(f"{name}/kernel"), z, act="lrelu", alpha=ALPHA, ws=ws, planes=P[l])
            else:
                y = s["yd"][l]
                d.fwd(h, A.param(f"{name}/kernel"), y, ws=ws, planes=P[l])
                # z feeds the next down conv (plane index l+1; down8's z8 feeds
                # up1, index 8) and, as the skip half of cat[6-l], the up conv
                # reading that concat (index 15-l, its columns after up 6-l's) -- bf16x6
                # planes there; fp16x3 concat planes are written by up 6-l's BN, one scale
                # over both halves (below)
                nxt = l + 1
                outs = [(nxt, co, 0)] if xplanes(nxt) is not None else []
                if 1 <= l <= 6 and xplanes(15 - l) is not None and not (ab is not None and x3_planes(P[15 - l])):
                    outs.append((15 - l, self.ups[7 - l][1], self.ups[6 - l][2]))
                self._bn_fwd(s, name, y, z, "lrelu", training, ws, outs=outs,
                             z_bound=ab.zb[l] if ab is not None else None)
                if xplanes(nxt) is not None:
                    P[nxt]._filled(ops.TENSOR_X)
            h = z
        for u, (name, ci, co, drop) in enumerate(self.ups):
            d = self.udesc[u]
            y = s["yu"][u]
            d.fwd(h, A.param(f"{name}/kernel"), y, ws=ws, planes=P[8 + u])
            z = s["cat"][u][..., :co]
            rate = drop_rate if (drop and training) else 0.0
            # z is the first half of cat[u], read by plane index 9+u (up u+1, or
            # last); its skip half came from down 6-u's BN above (down1 is a
            # conv: cat[6]'s planes are split by its consumer as before)
            k = 9 + u
            outs = []
            copy = None
            if u <= 5 and xplanes(k) is not None:
                outs.append((k, self.ups[u + 1][1], 0))
                if ab is not None and x3_planes(P[k]):   # (+ the skip half, down 6-u's output, under one bound)
                    copy = (self.z_view(s, 6 - u), co, ab.zb[6 - u])
            self._bn_fwd(s, name, y, z, "relu", training, ws, rate, lambda hv: dropout_seed(drop_seed, u, hv),
                         step_dev, outs=outs, z_bound=ab.zb[8 + u] if ab is not None else None, copy=copy)
            if outs:
                P[k]._filled(ops.TENSOR_X)
            h = s["cat"][u]
        self.ldesc.fwd(h, A.param("last/kernel"), out, bias=A.param("last/bias"), act="tanh", ws=ws, planes=P[15])
        return out

    def _fwd_planes(self):
        """The layer planes with x and w invalidated (a forward re-splits both)."""
        for p in self.planes:
            if p is not None:
                p.invalidate(ops.TENSOR_X | ops.TENSOR_W)
        return self.planes

    def _bwd_planes(self, i):
        p = self.planes[i]
        if p is not None:
            p.invalidate(ops.TENSOR_DY)
        return p

    def _bn_fwd(self, s, name, y, z, act, training, ws, drop_rate=0.0, seed_of=None, step_dev=None, outs=(),
                z_bound=None, copy=None):
        """outs: (plane index k, its x channel count, column) -- the BN output is
        also written into plane k's kept x planes at that column (training).
        Training: one segmented call, each half normalised by its own statistics
        and the moving averages updated half 0 then half 1 (the reference's
        two generator calls); dropout seeds follow dropout_seed(base, layer, half)."""
        A = self.arena
        if training:
            rows = z[..., 0].numel()
            zp = [zplanes(self.planes[k].x, rows, pc, col) for k, pc, col in outs]
            seed0 = seed_of(0) if seed_of else 0
            stride = ((seed_of(1) - seed0) & 0xFFFFFFFF) if (seed_of and self.halves > 1) else 0
            ops.bn_fwd_train(y, A.param(f"{name}/gamma"), A.param(f"{name}/beta"), s["mean"][name], s["inv"][name],
                             self.bn.mean[name], self.bn.var[name], z, act=act, alpha=ALPHA, momentum=BN_MOMENTUM,
                             eps=BN_EPS, drop_rate=drop_rate, drop_seed=seed0, step_dev=step_dev, ws=ws, z_planes=zp,
                             segments=self.halves, drop_seed_stride=stride, z_bound=z_bound, copy=copy)
            return
        for hv in range(self.halves):
            ops.bn_fwd_infer(self._half(y, hv), A.param(f"{name}/gamma"), A.param(f"{name}/beta"), self.bn.mean[name],
                             self.bn.var[name], self._half(z, hv), act=act, alpha=ALPHA, eps=BN_EPS)

    def _bn_bwd(self, s, name, dz, z, y, dy, act, beta, ws, drop_rate=0.0, P=None, k=None):
        """BN backward per half; the gamma/beta gradients of the halves accumulate.
        P: the consuming conv's ConvPlanes (plane index k) -- when it keeps dy planes,
        the BN backward writes them beside dy (no split pass before the conv's
        backward GEMMs; fp16x3 planes with their bound into the conv's scale source)
        and marks them ready."""
        A = self.arena
        feed = P is not None and P.dy is not None
        ops.bn_bwd(dz, z, y, A.param(f"{name}/gamma"), s["mean"][name], s["inv"][name], dy, A.grad_of(f"{name}/gamma"),
                   A.grad_of(f"{name}/beta"), act=act, alpha=ALPHA, drop_rate=drop_rate, beta=beta, ws=ws,
                   dy_planes=plane_rows(P.dy, dy, 0) if feed else None, segments=self.halves,
                   dy_fp32=not (feed and DY_PLANES_ONLY), dy_bound=self.gbound[k] if feed else None,
                   offset=A.param(f"{name}/beta") if BN_RZ else None)
        if feed:
            P._filled(ops.TENSOR_DY)

    # backward ---------------------------------------------------------------
    def backward(self, dout, slot=0, beta=0.0, ws=None, drop_rate=DROP_RATE, on_grads_ready=None):
        """dout: grad of the tanh output over all halves (NHWC view).  Weight
        grads go to the arena grad buffer: g = new + beta * g (summed over the
        halves).  `on_grads_ready(name)` is called after each layer's
        gradients are enqueued (bucketed all-reduce)."""
        s = self.s
        A = self.arena
        dl = self.ldesc
        dpre = self._dy(dl, dl.Cout)
        ops.act_bwd(dout, s["out"], dpre, "tanh")
        P = self._bwd_planes(15)
        dl.bwd_filter(s["cat"][6], dpre, A.grad_of("last/kernel"), dbias=A.grad_of("last/bias"), beta=beta, ws=ws,
                      planes=P)
        dl.bwd_data(dpre, A.param("last/kernel"), self.dcat[6], ws=ws, planes=P)
        if on_grads_ready:
            on_grads_ready("last")
        for u in range(6, -1, -1):
            name, ci, co, drop = self.ups[u]
            d = self.udesc[u]
            dy = self._dy(d, co)
            P = self._bwd_planes(8 + u)
            self._bn_bwd(s, name, self.dcat[u][..., :co], s["cat"][u][..., :co], s["yu"][u], dy, "relu", beta, ws,
                         drop_rate=drop_rate if drop else 0.0, P=P if FEED_DY else None, k=8 + u)
            hin = s["z8"] if u == 0 else s["cat"][u - 1]
            dhin = self.dz8 if u == 0 else self.dcat[u - 1]
            d.bwd_filter(hin, dy, A.grad_of(f"{name}/kernel"), beta=beta, ws=ws, planes=P)
            d.bwd_data(dy, A.param(f"{name}/kernel"), dhin, ws=ws, planes=P)
            if on_grads_ready:
                on_grads_ready(name)
        masked_sum = False
        for l in range(7, -1, -1):
            name, ci, co, bn = self.downs[l]
            d = self.ddesc[l]
            dz = self.dz_view(l)
            z = self.z_view(s, l)
            dy = self._dy(d, co)
            P = self._bwd_planes(l)
            if bn:
                self._bn_bwd(s, name, dz, z, s["yd"][l], dy, "lrelu", beta, ws, P=P if FEED_DY else None, k=l)
            elif masked_sum:
                dy = dz   # (down2's input gradient applied act' to the summed gradient)
            else:
                ops.act_bwd(dz, z, dy, "lrelu", ALPHA)
            hin = s["x"] if l == 0 else self.z_view(s, l - 1)
            d.bwd_filter(hin, dy, A.grad_of(f"{name}/kernel"), beta=beta, ws=ws, planes=P)
            masked_sum = False
            if l > 0:
                # accumulate into the skip-gradient already sitting in the concat grad buffer; into
                # a LeakyReLU block without BN (down1) with act' applied to the sum in the epilogue
                if MASK_DZ and not self.downs[l - 1][3] and d.op_arith("bwd_data") != "fp32":
                    d.bwd_data_masked_sum(dy, A.param(f"{name}/kernel"), self.dz_view(l - 1),
                                          self.z_view(s, l - 1), "lrelu", ALPHA, beta=1.0, ws=ws, planes=P)
                    masked_sum = True
                else:
                    d.bwd_data(dy, A.param(f"{name}/kernel"), self.dz_view(l - 1), beta=1.0, ws=ws, planes=P)
            if on_grads_ready:
                on_grads_ready(name)


def g_layout_order(width=1):
    """Arena layout = backward completion order: last, up7..up1, down8..down1."""
    downs, ups, last = g_layer_specs(width)
    order = ["last/kernel", "last/bias"]
    for name, ci, co, _ in reversed(ups):
        order += [f"{name}/kernel", f"{name}/gamma", f"{name}/beta"]
    for name, ci, co, bn in reversed(downs):
        order.append(f"{name}/kernel")
        if bn:
            order += [f"{name}/gamma", f"{name}/beta"]
    return order


def d_layout_order(width=1):
    order = ["last/kernel", "last/bias"]
    for name, ci, co, bn in reversed(d_layer_specs(width)[:-1]):
        order.append(f"{name}/kernel")
        if bn:
            order += [f"{name}/gamma", f"{name}/beta"]
    return order


# ---------------------------------------------------------------------------
# PatchGAN discriminator plan (pix2pix.py:194-220)
# ---------------------------------------------------------------------------
class DiscriminatorPlan:
    """PatchGAN schedule.  halves=2 batches D([x, y]) (half 0, real) and
    D([x, G(x)]) (half 1, fake) into one pass over 2N images: the convs run
    once over both, BatchNorm per half (the reference's two separate calls);
    the parameter backward of both passes is one backward over 2N rows (the
    gradients of the two calls sum), and the input-gradient-only backward of
    the fake half runs on N-image descriptors over views of the same
    buffers.  `inp` is the [halves*N, H, W, 6] input buffer."""

    def __init__(self, N, H, W, width, arena, bn_state, device, halves=1, train=True, conv_math=None):
        self.N, self.H, self.W = N, H, W
        self.halves = halves
        math_ = conv_math or P2P_MATH
        NT = N * halves
        self.arena, self.bn = arena, bn_state
        self.specs = d_layer_specs(width)

        def descs(n):
            out = []
            h, w = H, W
            for name, ci, co, _ in self.specs:
                if name.startswith("down"):
                    d = ConvDesc(n, h, w, ci, co, 4, 2, "same", math=math_)
                else:  # ZeroPadding2D() + Conv2D(k4, s1, 'valid') == explicit pad 1
                    d = ConvDesc(n, h, w, ci, co, 4, 1, (1, 1, 1, 1), math=math_)
                d.label = f"D.{name}"
                out.append(d)
                h, w = d.Ho, d.Wo
            return out

        self.desc = descs(NT)
        self.desc_half = descs(N) if (train and halves > 1) else self.desc
        self.out_shape = self.desc[-1].out_shape
        self.inp = _empty((NT, H, W, self.specs[0][1]), device)
        self.y = [(_empty(d.out_shape, device) if sp[3] else None) for d, sp in zip(self.desc, self.specs)]
        self.z = [_empty(d.out_shape, device) for d in self.desc[:-1]]
        self.logits = _empty(self.out_shape, device)
        self.mean = {sp[0]: _empty((halves, sp[2]), device) for sp in self.specs if sp[3]}   # [half, channel]
        self.inv = {sp[0]: _empty((halves, sp[2]), device) for sp in self.specs if sp[3]}
        if train:
            self.dz = [_empty(d.out_shape, device) for d in self.desc[:-1]]
            maxdy = max(d.N * d.Ho * d.Wo * d.Cout for d in self.desc)
            self.dy = _empty((maxdy,), device)
        # bf16x6 operand planes (see GeneratorPlan); the half-batch backward
        # shares the weight planes and splits its own dy
        if train:
            self.planes = ops.plan_planes(self.desc, device)
            # D.down1 (conv + LeakyReLU, no BN) writes D.down2's x planes in its epilogue
            if FEED_X and self.planes[1].x is not None:
                self.planes[0].fwd_out = self.planes[1].x
            # (the half-batch pass runs on another stream beside the full backward and reads its
            # weight planes with no event wait: it shares a layer's buffer only when the full
            # pass's FORWARD splits the weights -- ready before either backward is enqueued; a
            # layer whose weights the full pass splits first in a backward op gets a buffer of its
            # own, split by the half pass itself)
            wshare = [p.w if (p.w is not None and d.plane_mask[ops.OP_FWD] & ops.TENSOR_W) else None
                      for p, d in zip(self.planes, self.desc)]
            self.planes_half = (ops.plan_planes(self.desc_half, device, keep_x=False, wbufs=wshare)
                                if self.desc_half is not self.desc else self.planes)
            # one dy bound per layer for the full backward; the half-batch backward (the G path
            # through D(fake)) has its own bounds, dz and dy scratch, so the two backwards may run
            # concurrently on two streams (trainer.Pix2PixTrainer overlap)
            self.gbound = grad_bounds(self.desc, self.planes, device)
            self.gbound_h = list(self.gbound)
            # fp16x3 activation planes scaled from their producers' bounds (ActBounds): D.down1's
            # conv output from (max |input pair|, down1's weight bound), BN block i's output zb[i]
            self.ab = None
            if ACT_BOUNDS and any(x3_planes(P) for P in self.planes):
                self.ab = ActBounds(len(self.desc), device)
                for k, d in enumerate(self.desc):
                    if x3_planes(self.planes[k]):
                        d.set_act_scale(x=self.ab.first_src if k == 1 else self.ab.zb[k - 1])
                if x3_planes(self.planes[1]) and FEED_X:
                    self.desc[0].set_act_scale(y=self.ab.first_src)
            if self.desc_half is not self.desc:
                for i, (d, P) in enumerate(zip(self.desc_half, self.planes_half)):
                    if FEED_DY and P is not None and P.dy is not None and P.dy.fmt == ops.PLANES_F16X3:
                        self.gbound_h[i] = ops.max_slot(device=device)
                        d.set_grad_scale(dy_m=self.gbound_h[i])
                self.dz_h = [_empty(d.out_shape, device) for d in self.desc_half[:-1]]
                self.dy_h = _empty((max(d.N * d.Ho * d.Wo * d.Cout for d in self.desc_half),), device)
        else:
            self.planes = self.planes_half = [None] * len(self.desc)
            self.ab = None
        # G path (train_pix2pix.py:64): of dL/d D([inp, G(x)]) only the G(x) channels 3..5
        # are used, so that input gradient runs as a Cin-3 conv over down1's filter slice
        # w[:, :, 3:6, :] (copied per step) straight into dL/dG(x) (beta 1); per channel the
        # sum is the one the 6-channel op computes
        self.desc_g3 = None
        if train and halves > 1 and self.specs[0][1] == 6:
            co1 = self.specs[0][2]
            self.desc_g3 = ConvDesc(N, H, W, 3, co1, 4, 2, "same")
            self.desc_g3.label = "D.down1.g"
            self.w_g3 = _empty((4, 4, 3, co1), device)
        self.ws_bytes = max([d.max_ws() for d in self.desc + self.desc_half] +
                            ([self.desc_g3.max_ws()] if self.desc_g3 is not None else []) +
                            [ops.bn_workspace_bytes(N * d.Ho * d.Wo, d.Cout, halves) for d in self.desc])

    @property
    def slots(self):
        return [{"inp": self.inp, "logits": self.logits}]

    def _half(self, t, h):
        return t[h * self.N:(h + 1) * self.N]

    def _dy(self, d, buf=None):
        buf = self.dy if buf is None else buf
        return buf[: d.N * d.Ho * d.Wo * d.Cout].view(d.N, d.Ho, d.Wo, d.Cout)

    def forward(self, slot=0, training=True, ws=None):
        A = self.arena
        h = self.inp
        for p in self.planes:
            if p is not None:
                p.invalidate(ops.TENSOR_X | ops.TENSOR_W)
        if self.planes_half is not self.planes:
            # (the half-batch backward shares a layer's weight planes only where its descriptor
            # has the same plane layout; a buffer of its own is split by its bwd_data)
            for p in self.planes_half:
                if p is not None:
                    p.invalidate(ops.TENSOR_W)
        ab = self.ab
        if ab is not None:
            ab.first_conv(self.inp, A.param("down1/kernel"))   # D.down2's x planes: (max |inp|, down1's bound)
        for i, (name, ci, co, bn) in enumerate(self.specs):
            d = self.desc[i]
            P = self.planes[i]
            if name == "last":
                d.fwd(h, A.param("last/kernel"), self.logits, bias=A.param("last/bias"), ws=ws, planes=P)
                return self.logits
            z = self.z[i]
            if not bn:
                d.fwd(h, A.param(f"{name}/kernel"), z, act="lrelu", alpha=ALPHA, ws=ws, planes=P)
            else:
                y = self.y[i]
                d.fwd(h, A.param(f"{name}/kernel"), y, ws=ws, planes=P)
                # z feeds the next conv's kept x planes (training)
                Pn = self.planes[i + 1]
                xp = Pn.x if FEED_X and training and Pn is not None else None
                if training:   # one segmented call: real and fake normalised separately, moving stats in order
                    rows = z[..., 0].numel()
                    ops.bn_fwd_train(y, A.param(f"{name}/gamma"), A.param(f"{name}/beta"), self.mean[name],
                                     self.inv[name], self.bn.mean[name], self.bn.var[name], z, act="lrelu",
                                     alpha=ALPHA, momentum=BN_MOMENTUM, eps=BN_EPS, ws=ws,
                                     z_planes=[zplanes(xp, rows, co, 0)] if xp is not None else (),
                                     segments=self.halves, z_bound=ab.zb[i] if ab is not None else None)
                else:
                    for hv in range(self.halves):
                        ops.bn_fwd_infer(self._half(y, hv), A.param(f"{name}/gamma"), A.param(f"{name}/beta"),
                                         self.bn.mean[name], self.bn.var[name], self._half(z, hv), act="lrelu",
                                         alpha=ALPHA, eps=BN_EPS)
                if xp is not None:
                    Pn._filled(ops.TENSOR_X)
            h = z

    def backward(self, dlogits, slot=0, param_grads=True, beta=0.0, input_grad=None, input_beta=0.0, ws=None,
                 on_grads_ready=None, half=None, input_from=0):
        """Backward through D.  half=None: over all halves (dlogits [halves*N]);
        half=h: over that half only (dlogits [N]), e.g. the G-path gradient
        through D(fake).  param_grads: accumulate weight grads (g = new +
        beta*g, summed over the halves covered); input_grad: NHWC view
        receiving dL/d(input) (+input_beta*old); input_from=3: only the
        input channels 3..5 (the generator output), input_grad has 3 channels."""
        A = self.arena
        hs = range(self.halves) if half is None else [half]
        desc = self.desc if half is None else self.desc_half

        def sub(t):  # the rows of t this pass covers
            return t if half is None else self._half(t, half)

        planes = self.planes if half is None else self.planes_half
        # (the half-batch pass has its own dz / dy scratch and dy bounds when built: it may run
        # on another stream beside the full pass)
        own = half is not None and getattr(self, "dz_h", None) is not None
        dzs = self.dz_h if own else self.dz
        dybuf = self.dy_h if own else None
        gb = self.gbound_h if own else self.gbound
        dh = dlogits
        masked = False   # dh already carries act'(z) of this layer's LeakyReLU (see bwd_data_masked below)
        n = len(self.specs)
        for i in range(n - 1, -1, -1):
            name, ci, co, bn = self.specs[i]
            d = desc[i]
            P = planes[i]
            if P is not None:
                P.invalidate(ops.TENSOR_DY)
            if name == "last":
                dy = dh
                if param_grads:
                    d.bwd_filter(sub(self.z[i - 1]), dy, A.grad_of("last/kernel"), dbias=A.grad_of("last/bias"),
                                 beta=beta, ws=ws, planes=P)
            else:
                dy = self._dy(d, dybuf)
                if bn:
                    feed = FEED_DY and P is not None and P.dy is not None
                    # all halves in one segmented call, or the one half's statistics
                    mean = self.mean[name] if half is None else self.mean[name][half]
                    inv = self.inv[name] if half is None else self.inv[name][half]
                    ops.bn_bwd(dh, sub(self.z[i]), sub(self.y[i]), A.param(f"{name}/gamma"), mean, inv, dy,
                               A.grad_of(f"{name}/gamma") if param_grads else None,
                               A.grad_of(f"{name}/beta") if param_grads else None, act="lrelu", alpha=ALPHA,
                               beta=beta, ws=ws, dy_planes=plane_rows(P.dy, dy, 0) if feed else None,
                               segments=len(hs), dy_fp32=not (feed and DY_PLANES_ONLY),
                               dy_bound=gb[i] if feed else None,
                               offset=A.param(f"{name}/beta") if BN_RZ else None)
                    if feed:
                        P._filled(ops.TENSOR_DY)
                elif masked:
                    dy = dh
                else:
                    ops.act_bwd(dh, sub(self.z[i]), dy, "lrelu", ALPHA)
                if param_grads:
                    hin = sub(self.inp) if i == 0 else sub(self.z[i - 1])
                    d.bwd_filter(hin, dy, A.grad_of(f"{name}/kernel"), beta=beta, ws=ws, planes=P)
            if param_grads and on_grads_ready:
                on_grads_ready(name)
            if i > 0:
                dz = dzs[i - 1] if own else sub(self.dz[i - 1])
                # a LeakyReLU block without BN below (down1, pix2pix.py:118-121): its act' applied
                # in this input gradient's epilogue -- no separate act_bwd pass over dz
                masked = MASK_DZ and not self.specs[i - 1][3]
                if masked:
                    d.bwd_data_masked(dy, A.param(f"{name}/kernel"), dz, sub(self.z[i - 1]), "lrelu", ALPHA, ws=ws,
                                      planes=P)
                else:
                    d.bwd_data(dy, A.param(f"{name}/kernel"), dz, ws=ws, planes=P)
                dh = dz
            elif input_grad is not None and input_from == 3:
                co = self.specs[0][2]
                ops.strided_copy(A.param(f"{name}/kernel").view(16, 6 * co)[:, 3 * co:], self.w_g3.view(16, 3 * co))
                self.desc_g3.bwd_data(dy, self.w_g3, input_grad, beta=input_beta, ws=ws)
            elif input_grad is not None:
                d.bwd_data(dy, A.param(f"{name}/kernel"), input_grad, beta=input_beta, ws=ws, planes=P)
