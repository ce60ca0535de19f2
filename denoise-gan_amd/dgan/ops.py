"""Tensor-level wrappers over the libdgan C ABI.

Tensors are torch CUDA (HIP) tensors used purely as device memory: NHWC,
fp32, last dim contiguous; a channel slice of a wider buffer is passed with
its pixel stride (zero-copy concat).  Every call enqueues on the current
torch stream and never synchronises.
"""
import ctypes

import torch

from ._lib import call, lib, DGError

# floats of a measured-max slot (include/dgan.h DG_MAX_SLOT: 8 atomic shards on their own
# 128-byte lines; tests/test_lib.py checks it against dg_max_slot_floats)
MAX_SLOT = 256


def max_slot(*lead, device=None):
    """A zeroed measured-max slot (or [*lead] of them): the fp16x3 scale sources' form."""
    return torch.zeros(*lead, MAX_SLOT, dtype=torch.float32, device=device)


ACT = {"none": 0, "linear": 0, None: 0, "lrelu": 1, "leaky_relu": 1, "relu": 2, "tanh": 3, "sigmoid": 4}
OP_FWD, OP_BWD_DATA, OP_BWD_FILTER = 0, 1, 2


def act_id(a):
    if isinstance(a, int):
        return a
    if a not in ACT:
        raise ValueError(f"unknown activation {a!r}")
    return ACT[a]


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def pix_ld(t, C=None):
    """Pixel stride (floats) of an NHWC (or [pixels, C]) view with contiguous channels."""
    if t.dtype != torch.float32:
        raise DGError(f"expected float32 tensor, got {t.dtype}")
    if not t.is_cuda:
        raise DGError("expected a device tensor (the HIP path has no CPU fallback)")
    if t.dim() not in (2, 4):
        raise DGError(f"expected NHWC or [pixels, C] tensor, got shape {tuple(t.shape)}")
    Cc = t.shape[-1]
    if Cc > 1 and t.stride(-1) != 1:
        raise DGError("channel dim must be contiguous")
    ld, expect = None, None
    for d in range(t.dim() - 2, -1, -1):  # pixel dims, innermost first
        size, st = t.shape[d], t.stride(d)
        if size == 1:
            continue
        if ld is None:
            ld = st
        elif st != expect:
            raise DGError(f"pixels of the view are not uniformly strided: shape {tuple(t.shape)} strides {t.stride()}")
        expect = st * size
    if ld is None:
        ld = Cc
    if C is not None and ld < C:
        raise DGError("pixel stride smaller than channel count")
    return ld


def tf_same_pads(size, k, s):
    """TF 'SAME' padding (before, after) for one spatial dim."""
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


class Workspace:
    """Grow-only device scratch shared by ops issued on one stream."""

    def __init__(self, device=None):
        self.device = device
        self.buf = None

    def get(self, nbytes):
        if nbytes == 0:
            return None, 0
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=self.device or "cuda")
        return self.buf, self.buf.numel()


_default_ws = {}


def default_conv_math():
    """The conv arithmetic new descriptors get (DG_CONV_MATH, default bf16x6)."""
    return ConvDesc(1, 8, 8, 16, 16, 3, 1, "same").math


def default_workspace():
    dev = torch.cuda.current_device()
    if dev not in _default_ws:
        _default_ws[dev] = Workspace(torch.device("cuda", dev))
    return _default_ws[dev]


# conv GEMM arithmetic (include/dgan.h DG_MATH_*)
MATH_FP32, MATH_BF16X6, MATH_FP16, MATH_F16X3 = 0, 1, 2, 3
MATH_MODES = {"fp32": MATH_FP32, "bf16x6": MATH_BF16X6, "fp16": MATH_FP16, "f16x3": MATH_F16X3}
# plane buffer formats (include/dgan.h DG_PLANES_*)
PLANES_BF16X6, PLANES_F16X3 = 0, 1

# layer tensors of dg_conv_planes_t (include/dgan.h DG_TENSOR_*)
TENSOR_X, TENSOR_DY, TENSOR_W = 1, 2, 4


class _PlanesC(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("dy", ctypes.c_void_p), ("w", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("ready", ctypes.c_int), ("out_format", ctypes.c_int)]


class PlaneBuf:
    """A device buffer of operand planes and whether it holds the split of the
    tensor it stands for.  One PlaneBuf may serve several ConvPlanes: the
    weight planes of a network read by several plans, or one output-gradient
    scratch reused layer after layer.  fmt: PLANES_BF16X6, or PLANES_F16X3 for
    the planes of a tensor that fp16x3 ops read (dg_conv_planes_format; a producer
    writing them needs to know).  layout: (format, bytes) of the descriptor that
    sized it -- a weight buffer is shared only between descriptors of the same
    layout (a bf16x6 [6 B], fp16x3 [4 B] and fp16x3 + bf16x6 [4 + 6 B] weight
    buffer hold different bytes at the same offsets).  stamp: the weight version
    its planes were split from (frozen networks keep them across forwards)."""

    __slots__ = ("buf", "ready", "fmt", "layout", "stamp")

    def __init__(self, nbytes, device=None, fmt=PLANES_BF16X6):
        self.buf = torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device or "cuda")
        self.ready = False
        self.fmt = fmt
        self.layout = (fmt, int(nbytes))
        self.stamp = None

    @classmethod
    def over(cls, t, layout):
        """A PlaneBuf over existing device bytes t (e.g. a view into a network's fp16 arena)."""
        v = cls.__new__(cls)
        v.buf, v.ready, v.fmt, v.layout, v.stamp = t, False, layout[0], layout, None
        return v

    def view(self, nbytes):
        """A PlaneBuf sharing the first nbytes of this one (own ready flag)."""
        v = PlaneBuf.__new__(PlaneBuf)
        v.buf, v.ready, v.fmt = self.buf[:max(int(nbytes), 16)], False, self.fmt
        v.layout, v.stamp = (self.fmt, int(nbytes)), None
        return v


def weight_layout(d):
    """(format, bytes) of descriptor d's weight planes: the key under which plans of one
    network may share a weight-plane buffer."""
    return (d.plane_format(TENSOR_W), d.plane_bytes(TENSOR_W))


class ConvPlanes:
    """Caller-held bf16x6 planes of one conv layer's tensors (dg_conv_planes_t).

    x / dy / w: PlaneBuf or None.  A conv wrapper called with planes marks
    a buffer ready after its op split that tensor into it; callers
    `invalidate` the tensors that change -- a new forward input or weights,
    a new output gradient.  out: the consumer's PlaneBuf for this layer's
    output (fwd) or input gradient (bwd_data); the op writes it beside the
    fp32 tensor and marks it ready (`fwd_out` / `bwd_out`)."""

    __slots__ = ("x", "dy", "w", "fwd_out", "bwd_out")

    def __init__(self, x=None, dy=None, w=None, fwd_out=None, bwd_out=None):
        self.x, self.dy, self.w = x, dy, w
        self.fwd_out, self.bwd_out = fwd_out, bwd_out

    @classmethod
    def for_desc(cls, d, x=False, dy=False, w=False, device=None):
        """Fresh buffers for the tensors of descriptor d that are asked for and
        that at least one op of d reads as planes."""
        used = d.plane_mask[0] | d.plane_mask[1] | d.plane_mask[2]

        def buf(t, want):
            return PlaneBuf(d.plane_bytes(t), device, d.plane_format(t)) if want and (used & t) else None

        return cls(buf(TENSOR_X, x), buf(TENSOR_DY, dy), buf(TENSOR_W, w))

    def _bufs(self):
        return ((TENSOR_X, self.x), (TENSOR_DY, self.dy), (TENSOR_W, self.w))

    @property
    def ready(self):
        return sum(t for t, b in self._bufs() if b is not None and b.ready)

    def invalidate(self, bits):
        for t, b in self._bufs():
            if b is not None and (bits & t):
                b.ready = False

    def _filled(self, bits):
        for t, b in self._bufs():
            if b is not None and (bits & t):
                b.ready = True

    def _c(self, out=None):
        ptr = lambda b: None if b is None else b.buf.data_ptr()
        return _PlanesC(ptr(self.x), ptr(self.dy), ptr(self.w), ptr(out), self.ready,
                        out.fmt if out is not None else PLANES_BF16X6)

    def _have(self):
        return sum(t for t, b in self._bufs() if b is not None)


def plan_planes(descs, device=None, keep_x=True, wbufs=None):
    """One ConvPlanes per descriptor of a training schedule (forward, then
    per layer bwd_filter -> bwd_data):
      x  -- its own buffer per layer, split by fwd and kept for bwd_filter
            (when both read x as planes and keep_x);
      w  -- split by fwd, reused by bwd_data (wbufs[i]: a PlaneBuf shared
            with other plans of the same weights);
      dy -- one scratch shared by all layers, split by bwd_filter, reused by
            bwd_data of the same layer.
    The schedule invalidates x and w before each fwd and dy before each
    layer's backward."""
    masks = [d.plane_mask for d in descs]
    dy_need = [d.plane_bytes(TENSOR_DY) if (m[1] & m[2] & TENSOR_DY) else 0 for d, m in zip(descs, masks)]
    dy_buf = PlaneBuf(max(dy_need), device) if dy_need and max(dy_need) else None
    out = []
    for i, (d, m) in enumerate(zip(descs, masks)):
        x = PlaneBuf(d.plane_bytes(TENSOR_X), device, d.plane_format(TENSOR_X)) if keep_x and (m[0] & m[2] & TENSOR_X) \
            else None
        w = None
        if (m[0] | m[1]) & TENSOR_W:
            # (a shared buffer only when its layout is this descriptor's: plans of one network
            # at different batch / image sizes may run a layer in different arithmetics)
            w = wbufs[i] if wbufs is not None else None
            if w is None or w.layout != weight_layout(d):
                w = PlaneBuf(d.plane_bytes(TENSOR_W), device, d.plane_format(TENSOR_W))
        dy = dy_buf.view(dy_need[i]) if dy_need[i] else None
        if dy is not None:
            dy.fmt = d.plane_format(TENSOR_DY)
        out.append(ConvPlanes(x, dy, w))
    return out


class ConvDesc:
    """A Conv2D / Conv2DTranspose layer geometry (immutable), libdgan descriptor.

    padding: 'same' | 'valid' | (top, bottom, left, right).  For transposed
    layers the pads are those of the equivalent forward conv, computed from
    the output size the way TF's conv2d_transpose does.
    """

    def __init__(self, N, H, W, Cin, Cout, kernel, strides=1, padding="same", transpose=False, math=None):
        kh, kw = (kernel, kernel) if isinstance(kernel, int) else kernel
        sh, sw = (strides, strides) if isinstance(strides, int) else strides
        if transpose:
            if padding == "same":
                Ho, Wo = H * sh, W * sw
            elif padding == "valid":
                Ho, Wo = H * sh + max(kh - sh, 0), W * sw + max(kw - sw, 0)
            else:
                pt, pb, pl, pr = padding
                Ho, Wo = (H - 1) * sh + kh - pt - pb, (W - 1) * sw + kw - pl - pr
            if padding in ("same", "valid"):
                th = max((H - 1) * sh + kh - Ho, 0)
                tw = max((W - 1) * sw + kw - Wo, 0)
                pt, pb, pl, pr = th // 2, th - th // 2, tw // 2, tw - tw // 2
        else:
            if padding == "same":
                pt, pb = tf_same_pads(H, kh, sh)
                pl, pr = tf_same_pads(W, kw, sw)
            elif padding == "valid":
                pt = pb = pl = pr = 0
            else:
                pt, pb, pl, pr = padding
        self.N, self.H, self.W, self.Cin, self.Cout = N, H, W, Cin, Cout
        self.kh, self.kw, self.sh, self.sw = kh, kw, sh, sw
        self.pads = (pt, pb, pl, pr)
        self.transpose = bool(transpose)
        h = ctypes.c_void_p()
        call("dg_conv_desc_create", ctypes.byref(h), N, H, W, Cin, Cout, kh, kw, sh, sw, pt, pb, pl, pr,
             int(self.transpose))
        self._h = h
        ho, wo = ctypes.c_int(), ctypes.c_int()
        call("dg_conv_out_shape", h, ctypes.byref(ho), ctypes.byref(wo))
        self.Ho, self.Wo = ho.value, wo.value
        if math is not None:
            call("dg_conv_set_math", h, MATH_MODES[math] if isinstance(math, str) else int(math))
        m = ctypes.c_int()
        call("dg_conv_get_math", h, ctypes.byref(m))
        self.math = m.value
        self.ws = []
        self.plane_mask = []   # per op: TENSOR_* bits it reads as bf16x6 planes
        for op in (OP_FWD, OP_BWD_DATA, OP_BWD_FILTER):
            n = ctypes.c_size_t()
            call("dg_conv_workspace_size", h, op, ctypes.byref(n))
            self.ws.append(n.value)
            m = ctypes.c_int()
            call("dg_conv_op_planes", h, op, ctypes.byref(m))
            self.plane_mask.append(m.value)

    def plane_bytes(self, tensor):
        n = ctypes.c_size_t()
        call("dg_conv_planes_size", self._h, tensor, ctypes.byref(n))
        return n.value

    def set_grad_scale(self, dy_m=None, dy_g=None, dx_m=None, dx_g=None, dx_max=None):
        """The fp16x3 input-gradient scale context (include/dgan.h dg_conv_set_grad_scale):
        device floats (views that stay alive with the plan; the measured maxima dy_m, dx_m and
        dx_max max slots), None = unset."""
        for t in (dy_m, dx_m, dx_max):
            if t is not None and t.numel() < MAX_SLOT:
                raise DGError(f"a measured gradient max is a max slot of {MAX_SLOT} floats (per-workgroup shards)")
        self._gs = (dy_m, dy_g, dx_m, dx_g, dx_max)   # (keeps the views referenced)
        call("dg_conv_set_grad_scale", self._h, _p(dy_m), _p(dy_g), _p(dx_m), _p(dx_g), _p(dx_max))

    def set_act_scale(self, x=None, y=None, y_max=None):
        """The fp16x3 activation scale context (include/dgan.h dg_conv_set_act_scale): x, y = (m, g, c)
        scale sources of the input planes and of the output planes the forward writes (device
        floats: m a max slot, g and c one float or None), y_max a max slot receiving max |y|."""
        def src(v):   # a tensor alone = (m,): a plain max slot
            v = (v,) if isinstance(v, torch.Tensor) else tuple(v or ())
            return v + (None,) * (3 - len(v))
        xs, ys = src(x), src(y)
        for t in (xs[0], ys[0], y_max):
            if t is not None and t.numel() < MAX_SLOT:
                raise DGError(f"a measured max / bound slot is {MAX_SLOT} floats (per-workgroup shards)")
        self._as = (xs, ys, y_max)   # (keeps the views referenced)
        call("dg_conv_set_act_scale", self._h, *(_p(t) for t in xs), *(_p(t) for t in ys), _p(y_max))

    def op_arith(self, op):
        """'fp32' | 'bf16x6' | 'fp16' | 'f16x3': the arithmetic of op's GEMM (dg_conv_op_arith)."""
        if isinstance(op, str):
            op = {"fwd": OP_FWD, "bwd_data": OP_BWD_DATA, "bwd_filter": OP_BWD_FILTER}[op]
        a = ctypes.c_int()
        call("dg_conv_op_arith", self._h, op, ctypes.byref(a))
        return ("fp32", "bf16x6", "fp16", "f16x3")[a.value]

    def plane_format(self, tensor):
        """PLANES_F16X3 for the x / w planes of a descriptor whose forward runs fp16x3."""
        f = ctypes.c_int()
        call("dg_conv_planes_format", self._h, tensor, ctypes.byref(f))
        return f.value

    def _pl(self, op, planes):
        """(struct pointer, bits this op fills) for a ConvPlanes (None -> no planes)."""
        if planes is None:
            return None, 0
        out = planes.fwd_out if op == OP_FWD else (planes.bwd_out if op == OP_BWD_DATA else None)
        if not self.plane_mask[op] and out is None:
            return None, 0
        st = planes._c(out)
        return ctypes.byref(st), self.plane_mask[op] & planes._have()

    def __del__(self):
        try:
            if getattr(self, "_h", None) is not None:
                lib().dg_conv_desc_destroy(self._h)
        except Exception:
            pass

    @property
    def out_shape(self):
        return (self.N, self.Ho, self.Wo, self.Cout)

    @property
    def weight_shape(self):
        return (self.kh, self.kw, self.Cout, self.Cin) if self.transpose else (self.kh, self.kw, self.Cin, self.Cout)

    def max_ws(self):
        return max(self.ws)

    def _ws(self, op, ws):
        ws = ws or default_workspace()
        buf, n = ws.get(self.ws[op])
        return (_p(buf), n)

    @property
    def flops(self):
        """Algorithmic FLOPs of one fwd / bwd_data / bwd_filter call (2 * MACs of the dense conv)."""
        if self.transpose:
            return 2 * self.N * self.H * self.W * self.Cin * self.kh * self.kw * self.Cout
        return 2 * self.N * self.Ho * self.Wo * self.Cout * self.kh * self.kw * self.Cin

    def op_bytes(self, op):
        """Algorithmic HBM bytes of one call: each fp32 operand read once, the output written once."""
        xin = self.N * self.H * self.W * self.Cin
        yout = self.N * self.Ho * self.Wo * self.Cout
        w = self.kh * self.kw * self.Cin * self.Cout
        return 4 * (xin + yout + w)

    # planes: optional ConvPlanes (bf16x6 operand planes shared between the
    # ops of this layer, include/dgan.h dg_conv_planes_t)
    def fwd(self, x, w, y, bias=None, act="none", alpha=0.3, beta=0.0, ws=None, planes=None):
        """y None: only the output's planes (planes.fwd_out) are written."""
        ldx, ldy = pix_ld(x, self.Cin), (pix_ld(y, self.Cout) if y is not None else 0)
        wp, wn = self._ws(OP_FWD, ws)
        pp, fills = self._pl(OP_FWD, planes)
        ev = _prof_begin()
        call("dg_conv_fwd_pl", self._h, _p(x), ldx, _p(w), _p(bias), _p(y), ldy,
             float(beta), act_id(act), float(alpha), pp, wp, wn, _stream())
        _prof_end(ev, self, "fwd")
        if fills:
            planes._filled(fills)
        if planes is not None and planes.fwd_out is not None:
            planes.fwd_out.ready = True
        return y

    def pool_fusable(self, act):
        """Whether fwd_pool can run MaxPool2D(2) in this layer's forward epilogue."""
        ok = ctypes.c_int()
        call("dg_conv_fwd_pool_ok", self._h, act_id(act), ctypes.byref(ok))
        return bool(ok.value)

    def fwd_pool(self, x, w, pool_idx, bias=None, act="none", alpha=0.3, pool_y=None, ws=None, planes=None,
                 pool_planes=None):
        """Conv forward + MaxPool2D(2) of its activated output in one epilogue
        (dg_conv_fwd_pool): the pooled values go to pool_y (may be None) and
        their bf16x6 planes to pool_planes (the next conv's x PlaneBuf);
        pool_idx [N, Ho/2, Wo/2, Cout] uint8 receives {argmax, value > 0} for
        maxpool2_bwd_idx.  The full-size activation is not written."""
        ldx = pix_ld(x, self.Cin)
        ldpy = pix_ld(pool_y, self.Cout) if pool_y is not None else 0
        wp, wn = self._ws(OP_FWD, ws)
        if planes is not None:
            saved, planes.fwd_out = planes.fwd_out, pool_planes
        pp, fills = self._pl(OP_FWD, planes)
        if planes is None and pool_planes is not None:
            pp, fills = ctypes.byref(_PlanesC(None, None, None, pool_planes.buf.data_ptr(), 0, pool_planes.fmt)), 0
        ev = _prof_begin()
        call("dg_conv_fwd_pool", self._h, _p(x), ldx, _p(w), _p(bias), act_id(act), float(alpha), _p(pool_y), ldpy,
             _p(pool_idx), pp, wp, wn, _stream())
        _prof_end(ev, self, "fwd")
        if planes is not None:
            planes.fwd_out = saved
            if fills:
                planes._filled(fills)
        if pool_planes is not None:
            pool_planes.ready = True
        return pool_y

    def bwd_data(self, dy, w, dx, beta=0.0, ws=None, planes=None):
        return self._bwd_data(dy, w, dx, None, 0, 0.0, beta, ws, planes)

    def bwd_data_masked(self, dy, w, dx, z, act, alpha=0.3, beta=0.0, ws=None, planes=None):
        """dx = dL/dx * act'(z) + beta*dx, z = the activation output this conv read as input."""
        return self._bwd_data(dy, w, dx, z, act_id(act), alpha, beta, ws, planes)

    def bwd_data_masked_sum(self, dy, w, dx, z, act, alpha=0.3, beta=1.0, ws=None, planes=None):
        """dx = act'(z) * (dL/dx + beta*dx): the mask also covers the gradient already in dx
        (dg_conv_bwd_data_masked_sum; split-precision plans only)."""
        lddy, lddx = pix_ld(dy, self.Cout), pix_ld(dx, self.Cin)
        wp, wn = self._ws(OP_BWD_DATA, ws)
        pp, fills = self._pl(OP_BWD_DATA, planes)
        ev = _prof_begin()
        call("dg_conv_bwd_data_masked_sum", self._h, _p(dy), lddy, _p(w), _p(dx), lddx, float(beta), _p(z),
             pix_ld(z, self.Cin), act_id(act), float(alpha), pp, wp, wn, _stream())
        _prof_end(ev, self, "bwd_data")
        if fills:
            planes._filled(fills)
        if planes is not None and planes.bwd_out is not None:
            planes.bwd_out.ready = True
        return dx

    def bwd_data_xmask(self, dy, w, dx, act, alpha=0.3, beta=0.0, ws=None, planes=None):
        """dx = dL/dx * act'(x) + beta*dx with act' from the sign of x's hi plane
        (planes.x, ready): the layer input need not exist in fp32."""
        lddy, lddx = pix_ld(dy, self.Cout), pix_ld(dx, self.Cin)
        wp, wn = self._ws(OP_BWD_DATA, ws)
        pp, fills = self._pl(OP_BWD_DATA, planes)
        if pp is None:
            pp, fills = ctypes.byref(planes._c(planes.bwd_out)), 0
        ev = _prof_begin()
        call("dg_conv_bwd_data_xmask", self._h, _p(dy), lddy, _p(w), _p(dx), lddx, float(beta), act_id(act),
             float(alpha), pp, wp, wn, _stream())
        _prof_end(ev, self, "bwd_data")
        if fills:
            planes._filled(fills)
        if planes.bwd_out is not None:
            planes.bwd_out.ready = True
        return dx

    def _bwd_data(self, dy, w, dx, z, act, alpha, beta, ws, planes):
        lddy, lddx = pix_ld(dy, self.Cout), pix_ld(dx, self.Cin)
        ldz = pix_ld(z, self.Cin) if z is not None else 0
        wp, wn = self._ws(OP_BWD_DATA, ws)
        pp, fills = self._pl(OP_BWD_DATA, planes)
        ev = _prof_begin()
        call("dg_conv_bwd_data_pl", self._h, _p(dy), lddy, _p(w), _p(dx), lddx, float(beta), _p(z), ldz, act,
             float(alpha), pp, wp, wn, _stream())
        _prof_end(ev, self, "bwd_data")
        if fills:
            planes._filled(fills)
        if planes is not None and planes.bwd_out is not None:
            planes.bwd_out.ready = True
        return dx

    def bwd_filter(self, x, dy, dw, dbias=None, beta=0.0, ws=None, planes=None):
        ldx, lddy = pix_ld(x, self.Cin), pix_ld(dy, self.Cout)
        wp, wn = self._ws(OP_BWD_FILTER, ws)
        pp, fills = self._pl(OP_BWD_FILTER, planes)
        ev = _prof_begin()
        call("dg_conv_bwd_filter_pl", self._h, _p(x), ldx, _p(dy), lddy, _p(dw),
             _p(dbias), float(beta), pp, wp, wn, _stream())
        _prof_end(ev, self, "bwd_filter")
        if fills:
            planes._filled(fills)
        return dw


# ---------------------------------------------------------------------------
# optional per-conv timing with HIP events on the launching stream (bench.py
# roofline leg); off unless a ConvProfile is active
# ---------------------------------------------------------------------------
_PROF = None


class ConvProfile:
    """Records (HIP start event, end event, desc, op) around every conv call.
    markers: also put a dg_mark dispatch before and after every conv call (and
    `mark()` wherever the caller wants one), so per-dispatch PMC counters can be
    attributed to conv calls (scripts/pmc_layers.py); `marks` lists them in order."""

    def __init__(self, markers=False):
        self.records = []
        self.markers = markers
        self.marks = []

    def mark(self, what):
        if self.markers:
            call("dg_mark", len(self.marks), _stream())
            self.marks.append(what)

    def __enter__(self):
        global _PROF
        self._prev, _PROF = _PROF, self
        return self

    def __exit__(self, *a):
        global _PROF
        _PROF = self._prev

    def summary(self):
        """-> list of dicts (op, shape, flops, ms); call after synchronising."""
        out = []
        for e0, e1, d, op in self.records:
            out.append(dict(op=op, label=getattr(d, "label", None), transpose=d.transpose,
                            shape=(d.N, d.H, d.W, d.Cin, d.Cout, d.kh, d.sh), arith=d.op_arith(op),
                            flops=d.flops, bytes=d.op_bytes(op), ms=e0.elapsed_time(e1)))
        return out


def profiling():
    """A ConvProfile is recording: callers run their work on one stream (per-op events on two
    concurrent streams would time the overlap, not the op)."""
    return _PROF is not None


def _prof_begin():
    if _PROF is None:
        return None
    _PROF.mark(("begin", len(_PROF.records)))
    e = torch.cuda.Event(enable_timing=True)
    e.record(torch.cuda.current_stream())
    return e


def _prof_end(e0, desc, op):
    if e0 is None:
        return
    e1 = torch.cuda.Event(enable_timing=True)
    e1.record(torch.cuda.current_stream())
    _PROF.mark(("end", len(_PROF.records)))
    _PROF.records.append((e0, e1, desc, op))


def bn_workspace_bytes(M, C, segments=1):
    n = ctypes.c_size_t()
    call("dg_bn_workspace_size_seg", segments, M, C, ctypes.byref(n))
    return n.value


def _rows(t):
    return t.numel() // t.shape[-1] if t.dim() == 2 else t.shape[0] * t.shape[1] * t.shape[2]


def bn_fwd_train(y, gamma, beta, save_mean, save_invstd, moving_mean, moving_var, z, act="none", alpha=0.3,
                 momentum=0.99, eps=1e-3, drop_rate=0.0, drop_seed=0, step_dev=None, ws=None, z_planes=(),
                 segments=1, drop_seed_stride=0, f16_out=None, res=None, z_bound=None, copy=None):
    """z_planes: up to two (uint8 device tensor, planes C, column) -- packed x
    planes of consuming convs that also receive z.  segments: the rows are that
    many consecutive independent BN calls (dg_bn_fwd_train_seg; save_mean /
    save_invstd [segments, C], dropout seed drop_seed + s * drop_seed_stride).
    f16_out: the consuming fp16 conv's x PlaneBuf, which also receives z's fp16 copy.
    res: a residual Add fused after the block, z = act(BN(y)) + res (same shape as z).
    z_bound: 8 device floats, the bound of z that scales fp16x3 z planes (written here,
    dg_bn_fwd_train_seg_x; the consumers' x scale source).  copy: (tensor, column, its bound)
    -- a second tensor's planes into z_planes[0] at that column with the same scale (the
    U-Net skip half of a concatenation)."""
    if z_bound is not None or copy is not None:
        if res is not None or f16_out is not None:
            # (dg_bn_fwd_train_seg_x rejects a residual with a z bound; the fp16 copy is not routed)
            raise DGError("bn_fwd_train: z_bound / copy cannot be combined with res or f16_out")
        return _bn_fwd_train_x(y, gamma, beta, save_mean, save_invstd, moving_mean, moving_var, z, act, alpha,
                               momentum, eps, drop_rate, drop_seed, step_dev, ws, z_planes, segments,
                               drop_seed_stride, z_bound, copy)
    C = y.shape[-1]
    M = _rows(y)
    if M % segments:
        raise DGError(f"{M} rows do not split into {segments} segments")
    M //= segments
    ws = ws or default_workspace()
    buf, n = ws.get(bn_workspace_bytes(M, C, segments))
    zp = [(t.data_ptr(), int(pc), int(col)) for t, pc, col in z_planes] + [(None, 0, 0)] * (2 - len(z_planes))
    call("dg_bn_fwd_train_seg_h", segments, M, C, _p(y), pix_ld(y, C), _p(gamma), _p(beta), _p(save_mean),
         _p(save_invstd), _p(moving_mean), _p(moving_var), float(momentum), float(eps), _p(z), pix_ld(z, C),
         act_id(act), float(alpha), float(drop_rate), ctypes.c_uint32(drop_seed & 0xFFFFFFFF),
         ctypes.c_uint32(drop_seed_stride & 0xFFFFFFFF), _p(step_dev),
         zp[0][0], zp[0][1], zp[0][2], zp[1][0], zp[1][1], zp[1][2], _p(res), pix_ld(res, C) if res is not None else 0,
         _f16(f16_out), _p(buf), n, _stream())
    return z


def _bn_fwd_train_x(y, gamma, beta, save_mean, save_invstd, moving_mean, moving_var, z, act, alpha, momentum, eps,
                    drop_rate, drop_seed, step_dev, ws, z_planes, segments, drop_seed_stride, z_bound, copy):
    C = y.shape[-1]
    M = _rows(y)
    if M % segments:
        raise DGError(f"{M} rows do not split into {segments} segments")
    M //= segments
    if z_bound is None or z_bound.numel() < MAX_SLOT:
        raise DGError(f"a z bound is a max slot of {MAX_SLOT} device floats (per-workgroup shards)")
    ws = ws or default_workspace()
    buf, n = ws.get(bn_workspace_bytes(M, C, segments))
    zp = [(t.data_ptr(), int(pc), int(col)) for t, pc, col in z_planes] + [(None, 0, 0)] * (2 - len(z_planes))
    cp, cpcol, cpb = copy if copy is not None else (None, 0, None)
    cpC = cp.shape[-1] if cp is not None else 0
    call("dg_bn_fwd_train_seg_x", segments, M, C, _p(y), pix_ld(y, C), _p(gamma), _p(beta), _p(save_mean),
         _p(save_invstd), _p(moving_mean), _p(moving_var), float(momentum), float(eps), _p(z), pix_ld(z, C),
         act_id(act), float(alpha), float(drop_rate), ctypes.c_uint32(drop_seed & 0xFFFFFFFF),
         ctypes.c_uint32(drop_seed_stride & 0xFFFFFFFF), _p(step_dev),
         zp[0][0], zp[0][1], zp[0][2], zp[1][0], zp[1][1], zp[1][2], _p(z_bound),
         _p(cp), pix_ld(cp, cpC) if cp is not None else 0, cpC, int(cpcol), _p(cpb), None, 0, None, _p(buf), n,
         _stream())
    return z


def bn_fwd_infer(y, gamma, beta, moving_mean, moving_var, z, act="none", alpha=0.3, eps=1e-3):
    C = y.shape[-1]
    call("dg_bn_fwd_infer", _rows(y), C, _p(y), pix_ld(y, C), _p(gamma), _p(beta), _p(moving_mean),
         _p(moving_var), float(eps), _p(z), pix_ld(z, C), act_id(act), float(alpha), _stream())
    return z


def bn_bwd(dz, z, y, gamma, save_mean, save_invstd, dy, dgamma, dbeta, act="none", alpha=0.3, drop_rate=0.0,
           beta=0.0, ws=None, dy_planes=None, segments=1, dy_fp32=True, f16_out=None, dy_bound=None, offset=None):
    """dy_planes: a uint8 device tensor (e.g. a slice of a ConvPlanes' dy
    PlaneBuf) that also receives dy's bf16x6 planes -- or, with dy_bound (8 device
    floats, the consuming conv's dy scale source), its fp16x3 planes scaled from the
    bound written there (dg_bn_bwd_seg_x); dy_fp32=False then skips the fp32 dy (its
    consumers read the planes; dy only gives the shape).
    segments: see bn_fwd_train (dg_bn_bwd_seg; dgamma / dbeta summed over the
    segments).  f16_out: the producing fp16 conv's dy PlaneBuf (dy's fp16 copy).
    offset: the BN's beta (the forward's value): a ReLU / LeakyReLU block without dropout
    then recomputes act'(z) from y (dg_bn_bwd_seg_r) and z is not read (may be None)."""
    C = y.shape[-1]
    M = _rows(y)
    if M % segments:
        raise DGError(f"{M} rows do not split into {segments} segments")
    M //= segments
    ws = ws or default_workspace()
    buf, n = ws.get(bn_workspace_bytes(M, C, segments))
    if act_id(act) == 0 and drop_rate == 0.0:
        z = None   # a linear BN's backward does not read z (dg_bn_bwd_seg_h)
    if dy_bound is not None and dy_bound.numel() < MAX_SLOT:
        raise DGError(f"a gradient bound is a max slot of {MAX_SLOT} floats (per-workgroup shards)")
    if offset is not None and act_id(act) in (ACT["relu"], ACT["lrelu"]) and drop_rate == 0.0:
        call("dg_bn_bwd_seg_r", segments, M, C, _p(dz), pix_ld(dz, C), _p(y), pix_ld(y, C), _p(gamma), _p(offset),
             _p(save_mean), _p(save_invstd), act_id(act), float(alpha),
             _p(dy) if (dy_fp32 or dy_planes is None) else None, pix_ld(dy, C),
             None if dy_planes is None else dy_planes.data_ptr(),
             PLANES_F16X3 if dy_bound is not None else PLANES_BF16X6, _p(dy_bound), _f16(f16_out),
             _p(dgamma), _p(dbeta), float(beta), _p(buf), n, _stream())
        return dy
    call("dg_bn_bwd_seg_x", segments, M, C, _p(dz), pix_ld(dz, C), _p(z), pix_ld(z, C) if z is not None else C,
         _p(y), pix_ld(y, C),
         _p(gamma), _p(save_mean), _p(save_invstd), act_id(act), float(alpha), float(drop_rate),
         _p(dy) if (dy_fp32 or dy_planes is None) else None, pix_ld(dy, C),
         None if dy_planes is None else dy_planes.data_ptr(),
         PLANES_F16X3 if dy_bound is not None else PLANES_BF16X6, _p(dy_bound), _f16(f16_out),
         _p(dgamma), _p(dbeta), float(beta), _p(buf), n, _stream())
    return dy


def act_bwd(dz, z, dy, act, alpha=0.3):
    C = z.shape[-1]
    call("dg_act_bwd", _rows(z), C, _p(dz), pix_ld(dz, C), _p(z), pix_ld(z, C), act_id(act), float(alpha),
         _p(dy), pix_ld(dy, C), _stream())
    return dy


LOSS_WEIGHTS_REF = (1e-3, 1.0, 1.0, 1e-5, 1.0, 1.0)  # gan, l1, l2, tv, identity, content (pix2pix.py:75-92)


def p2p_loss_workspace_bytes(B, H, W, C, n_logits):
    n = ctypes.c_size_t()
    call("dg_p2p_loss_workspace_size", B, H, W, C, n_logits, ctypes.byref(n))
    return n.value


def p2p_loss(gen, tgt, logit_real, logit_fake, out, ident=None, weights=LOSS_WEIGHTS_REF, content=None,
             dgen=None, dident=None, dlogit_real_d=None, dlogit_fake_d=None, dlogit_fake_g=None, ws=None):
    B, H, W, C = gen.shape
    nlog = logit_fake.numel()
    ws = ws or default_workspace()
    buf, n = ws.get(p2p_loss_workspace_bytes(B, H, W, C, nlog))
    warr = (ctypes.c_float * 6)(*[float(v) for v in weights])
    call("dg_p2p_loss", B, H, W, C, _p(gen), pix_ld(gen, C), _p(tgt), pix_ld(tgt, C), _p(ident),
         pix_ld(ident, C) if ident is not None else C, _p(logit_real), _p(logit_fake), nlog, warr, _p(content),
         _p(out), _p(dgen), pix_ld(dgen, C) if dgen is not None else C, _p(dident),
         pix_ld(dident, C) if dident is not None else C, _p(dlogit_real_d), _p(dlogit_fake_d), _p(dlogit_fake_g),
         _p(buf), n, _stream())
    return out


def adam(p, g, m, v, lr, beta1, beta2, eps, iter_dev, grad_scale=1.0):
    call("dg_adam", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), float(beta1), float(beta2), float(eps),
         float(grad_scale), _p(iter_dev), _stream())


def scale_by(t, loss_scale):
    """t *= loss_scale[0] (contiguous device tensor; the dynamic loss scale's seed scaling)."""
    if not t.is_contiguous():
        raise DGError("scale_by needs a contiguous tensor")
    call("dg_scale_by", t.numel(), _p(t), _p(loss_scale), _stream())


def check_finite(g, loss_scale):
    call("dg_check_finite", g.numel(), _p(g), _p(loss_scale), _stream())


def adam_ls(p, g, m, v, lr, decay_steps, decay_rate, staircase, beta1, beta2, eps, iter_dev, loss_scale,
            grad_scale=1.0):
    call("dg_adam_ls", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), int(decay_steps), float(decay_rate),
         int(bool(staircase)), float(beta1), float(beta2), float(eps), float(grad_scale), _p(iter_dev),
         _p(loss_scale), _stream())


def counter_add_ls(c, loss_scale, inc=1):
    call("dg_counter_add_ls", _p(c), int(inc), _p(loss_scale), _stream())


def loss_scale_update(loss_scale, period=2000, multiplier=2.0):
    call("dg_loss_scale_update", _p(loss_scale), int(period), float(multiplier), _stream())


def counter_add(c, inc=1):
    call("dg_counter_add", _p(c), int(inc), _stream())


def channel_concat(a, b, out):
    ca, cb = a.shape[-1], b.shape[-1]
    npix = _rows(a)
    call("dg_channel_concat", npix, _p(a), pix_ld(a, ca), ca, _p(b), pix_ld(b, cb), cb, _p(out),
         pix_ld(out, ca + cb), _stream())
    return out


def to_f16(src, dst):
    """dst (float16, contiguous) = fp16(src) in one launch (dg_to_f16)."""
    if not (src.is_contiguous() and dst.is_contiguous()) or dst.numel() < src.numel():
        raise DGError("to_f16 needs contiguous tensors and room for every element")
    call("dg_to_f16", src.numel(), _p(src), dst.data_ptr(), _stream())
    return dst


def fill(t, value):
    if not t.is_contiguous():
        raise DGError("fill needs a contiguous tensor")
    call("dg_fill", _p(t), t.numel(), float(value), _stream())
    return t


def stage_pair(x, y, cat, catx=None, gx=None, gy=None):
    """One launch: cat = [x | y] along channels, catx[..., :C] = x, gx = x, gy = y (dg_stage_pair;
    x, y dense NHWC, gx / gy dense, catx / gx / gy optional)."""
    C = x.shape[-1]
    if y.shape != x.shape or not (x.is_contiguous() and y.is_contiguous()):
        raise DGError("stage_pair: x and y are dense tensors of one shape")
    pix_ld(x, C), pix_ld(y, C)
    for t, c in ((cat, 2 * C), (catx, C)):
        if t is not None and (_rows(t) != _rows(x) or t.shape[-1] < c):
            raise DGError("stage_pair: cat / catx have x's pixels and at least 2C / C channels")
    for t in (gx, gy):
        if t is not None and (t.shape != x.shape or not t.is_contiguous()):
            raise DGError("stage_pair: gx / gy are dense tensors of x's shape")
    call("dg_stage_pair", _rows(x), C, _p(x), _p(y), _p(cat), pix_ld(cat, 2 * C), _p(catx),
         pix_ld(catx, C) if catx is not None else 0, _p(gx), _p(gy), _stream())


def strided_copy(src, dst):
    C = src.shape[-1]
    call("dg_strided_copy", _rows(src), C, _p(src), pix_ld(src, C), _p(dst), pix_ld(dst, C), _stream())
    return dst


def adam_sched(p, g, m, v, lr, decay_steps, decay_rate, staircase, beta1, beta2, eps, iter_dev, grad_scale=1.0):
    """Keras Adam under ExponentialDecay(lr, decay_steps, decay_rate, staircase) (srgan.py:34-46)."""
    call("dg_adam_sched", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), int(decay_steps), float(decay_rate),
         int(bool(staircase)), float(beta1), float(beta2), float(eps), float(grad_scale), _p(iter_dev), _stream())


# ---------------------------------------------------------------------------
# SRGAN / FastSRGAN / Autoencoder / VGG19 layers (csrc/layers.hip)
# ---------------------------------------------------------------------------
def _nhwc(t):
    if t.dim() != 4:
        raise DGError(f"expected an NHWC tensor, got shape {tuple(t.shape)}")
    return t.shape


def prelu_workspace_bytes(N, H, W, C, block):
    n = ctypes.c_size_t()
    call("dg_prelu_workspace_size", N, H, W, C, block, ctypes.byref(n))
    return n.value


def _f16(buf):
    """Device pointer of an fp16 operand-copy destination (PlaneBuf or tensor), or None."""
    if buf is None:
        return None
    t = buf.buf if isinstance(buf, PlaneBuf) else buf
    return t.data_ptr()


def prelu_fwd(y, alpha, z, block=1, f16_out=None):
    """z = PReLU(depth_to_space(y, block)); y [N,H,W,C*block^2] -> z [N,H*block,W*block,C].
    f16_out: the consuming fp16 conv's x PlaneBuf, which also receives z's fp16 copy."""
    N, H, W, CB = _nhwc(y)
    C = CB // (block * block)
    call("dg_prelu_fwd_h", N, H, W, C, block, _p(y), pix_ld(y, CB), _p(alpha), _p(z), pix_ld(z, C), _f16(f16_out),
         _stream())
    return z


def prelu_bwd(y, alpha, dz, dy, dalpha=None, block=1, beta=0.0, alpha_beta=0.0, ws=None, f16_out=None):
    """f16_out: the producing fp16 conv's dy PlaneBuf, which also receives dy's fp16 copy."""
    N, H, W, CB = _nhwc(y)
    C = CB // (block * block)
    ws = ws or default_workspace()
    buf, n = ws.get(prelu_workspace_bytes(N, H, W, C, block))
    call("dg_prelu_bwd_h", N, H, W, C, block, _p(y), pix_ld(y, CB), _p(alpha), _p(dz), pix_ld(dz, C), _p(dy),
         pix_ld(dy, CB), _f16(f16_out), float(beta), _p(dalpha), float(alpha_beta), _p(buf), n, _stream())
    return dy


def add(a, b, out, f16_out=None):
    """f16_out: the consuming fp16 conv's x PlaneBuf, which also receives out's fp16 copy."""
    C = a.shape[-1]
    call("dg_add_h", _rows(a), C, _p(a), pix_ld(a, C), _p(b), pix_ld(b, C), _p(out), pix_ld(out, C), _f16(f16_out),
         _stream())
    return out


def accumulate(src, dst, beta=1.0):
    C = src.shape[-1]
    call("dg_accumulate", _rows(src), C, _p(src), pix_ld(src, C), _p(dst), pix_ld(dst, C), float(beta), _stream())
    return dst


def act_fwd(x, z, act, alpha=0.3):
    C = x.shape[-1]
    call("dg_act_fwd", _rows(x), C, _p(x), pix_ld(x, C), act_id(act), float(alpha), _p(z), pix_ld(z, C), _stream())
    return z


def maxpool2_fwd(x, y, planes_out=None, scale=None):
    """planes_out: PlaneBuf of the consuming conv's input planes, written beside y; scale: the
    (m, g, c) source of fp16x3 planes (the producing conv's output source, dg_maxpool2_fwd_x3)."""
    N, H, W, C = _nhwc(x)
    sm, sg, sc = scale if scale is not None else (None, None, None)
    call("dg_maxpool2_fwd_x3", N, H, W, C, _p(x), pix_ld(x, C), _p(y), pix_ld(y, C),
         None if planes_out is None else _p(planes_out.buf), PLANES_BF16X6 if planes_out is None else planes_out.fmt,
         _p(sm), _p(sg), _p(sc), _stream())
    if planes_out is not None:
        planes_out.ready = True
    return y


def maxpool2_bwd(x, dy, dx, beta=0.0, act="none", alpha=0.3, planes_out=None):
    """dx = routed dy * act'(x) + beta*dx (act: the activation whose output x is);
    planes_out: PlaneBuf of the producing conv's dy planes, written beside dx."""
    N, H, W, C = _nhwc(x)
    call("dg_maxpool2_bwd_pl", N, H, W, C, _p(x), pix_ld(x, C), _p(dy), pix_ld(dy, C), _p(dx), pix_ld(dx, C),
         float(beta), act_id(act), float(alpha), None if planes_out is None else _p(planes_out.buf), _stream())
    if planes_out is not None:
        planes_out.ready = True
    return dx


def maxpool2_bwd_idx(idx, dy, dx, C, H, W, beta=0.0, act="none", alpha=0.3, planes_out=None, scale=None):
    """Backward of a pool fused by ConvDesc.fwd_pool: dx [N,H,W,C] (may be None
    when planes_out, the producing conv's dy PlaneBuf, is all that is read).  scale:
    (m, g) device scalars (g may be None) -- the scale source of fp16x3 dy planes
    (include/dgan.h dg_conv_set_grad_scale); planes_out must then be an fp16x3 buffer."""
    N = dy.shape[0]
    sm, sg = scale if scale is not None else (None, None)
    if planes_out is not None and planes_out.fmt == PLANES_F16X3 and sm is None:
        raise DGError("fp16x3 gradient planes need a scale source")
    call("dg_maxpool2_bwd_idx_x3", N, H, W, C, _p(idx), _p(dy), pix_ld(dy, C), _p(dx),
         pix_ld(dx, C) if dx is not None else 0, float(beta), act_id(act), float(alpha),
         None if planes_out is None else _p(planes_out.buf), _p(sm), _p(sg), _stream())
    if planes_out is not None:
        planes_out.ready = True
    return dx


def absmax(t, out):
    """out (8 device floats, zeroed by the caller; the max is their max) = max(out, max |t|)
    (dg_absmax)."""
    if out.numel() < MAX_SLOT:
        raise DGError(f"absmax needs a max slot of {MAX_SLOT} floats (per-workgroup shards)")
    C = t.shape[-1]
    call("dg_absmax", _p(t), _rows(t), C, pix_ld(t, C), _p(out), _stream())
    return out


def absmax_set(t, out):
    """out (8 device floats) = max |t| (zeroed first, dg_absmax_set): a measured max."""
    if out.numel() < MAX_SLOT:
        raise DGError(f"absmax needs a max slot of {MAX_SLOT} floats (per-workgroup shards)")
    C = t.shape[-1]
    call("dg_absmax_set", _p(t), _rows(t), C, pix_ld(t, C), _p(out), _stream())
    return out


def weight_bound(w, g_out, bias=None, c_out=None, zero=None):
    """g_out[0] = max over output channels of sum |w| over the other axes (HWIO w), c_out[0] =
    max |bias| (dg_weight_bound): a conv output's bound terms; zero: a max slot zeroed on the way."""
    Co = w.shape[-1]
    call("dg_weight_bound", _p(w), w.numel() // Co, Co, _p(bias), _p(g_out), _p(c_out), _p(zero), _stream())


def weight_bound_in(w, g_out):
    """g_out[0] = max over input channels of sum |w| over the taps and output channels (HWIO w,
    dg_weight_bound_in): the weight term of an input gradient's bound."""
    kh, kw, Ci, Co = w.shape
    call("dg_weight_bound_in", _p(w), kh * kw, Ci, Co, _p(g_out), _stream())


def upsample2_relu_fwd(x, z):
    N, H, W, C = _nhwc(x)
    call("dg_upsample2_relu_fwd", N, H, W, C, _p(x), pix_ld(x, C), _p(z), pix_ld(z, C), _stream())
    return z


def upsample2_relu_bwd(x, dz, dx, beta=0.0):
    N, H, W, C = _nhwc(x)
    call("dg_upsample2_relu_bwd", N, H, W, C, _p(x), pix_ld(x, C), _p(dz), pix_ld(dz, C), _p(dx), pix_ld(dx, C),
         float(beta), _stream())
    return dx


def dwconv3_workspace_bytes(N, H, W, C):
    n = ctypes.c_size_t()
    call("dg_dwconv3_workspace_size", N, H, W, C, ctypes.byref(n))
    return n.value


def dwconv3_fwd(x, k, y, bias=None):
    N, H, W, C = _nhwc(x)
    call("dg_dwconv3_fwd", N, H, W, C, _p(x), pix_ld(x, C), _p(k), _p(bias), _p(y), pix_ld(y, C), _stream())
    return y


def dwconv3_bwd_data(dy, k, dx, beta=0.0):
    N, H, W, C = _nhwc(dy)
    call("dg_dwconv3_bwd_data", N, H, W, C, _p(dy), pix_ld(dy, C), _p(k), _p(dx), pix_ld(dx, C), float(beta),
         _stream())
    return dx


def dwconv3_bwd_filter(x, dy, dk, dbias=None, beta=0.0, ws=None):
    N, H, W, C = _nhwc(x)
    ws = ws or default_workspace()
    buf, n = ws.get(dwconv3_workspace_bytes(N, H, W, C))
    call("dg_dwconv3_bwd_filter", N, H, W, C, _p(x), pix_ld(x, C), _p(dy), pix_ld(dy, C), _p(dk), _p(dbias),
         float(beta), _p(buf), n, _stream())
    return dk


def vgg_preprocess_fwd(x, z):
    call("dg_vgg_preprocess_fwd", _rows(x), _p(x), pix_ld(x, 3), _p(z), pix_ld(z, 3), _stream())
    return z


def vgg_preprocess_bwd(dz, dx, beta=0.0):
    call("dg_vgg_preprocess_bwd", _rows(dz), _p(dz), pix_ld(dz, 3), _p(dx), pix_ld(dx, 3), float(beta), _stream())
    return dx


def mse_workspace_bytes():
    n = ctypes.c_size_t()
    call("dg_mse_workspace_size", ctypes.byref(n))
    return n.value


def mse(a, b, out, scale=1.0, da=None, grad_weight=1.0, ws=None):
    """out[0] = mean((scale*a - scale*b)^2); da = grad_weight * d out / d a."""
    C = a.shape[-1]
    ws = ws or default_workspace()
    buf, n = ws.get(mse_workspace_bytes())
    call("dg_mse", _rows(a), C, _p(a), pix_ld(a, C), _p(b), pix_ld(b, C), float(scale), _p(out), _p(da),
         pix_ld(da, C) if da is not None else C, float(grad_weight), _p(buf), n, _stream())
    return out


def gan_loss_workspace_bytes():
    n = ctypes.c_size_t()
    call("dg_gan_loss_workspace_size", ctypes.byref(n))
    return n.value


def gan_loss(gen, tgt, logit_real, logit_fake, out, coef, content=None, dgen=None, dlogit_real_d=None,
             dlogit_fake_d=None, dlogit_fake_g=None, ws=None):
    """coef = (w_adv, w_var, disc_scale, t_mae, t_mse, t_content, t_var); out[7] =
    (gen_total, adv, mae, mse, content, disc, var)."""
    B, H, W, C = gen.shape
    ws = ws or default_workspace()
    buf, n = ws.get(gan_loss_workspace_bytes())
    carr = (ctypes.c_float * 7)(*[float(v) for v in coef])
    call("dg_gan_loss", B, H, W, C, _p(gen), pix_ld(gen, C), _p(tgt), pix_ld(tgt, C), _p(logit_real),
         _p(logit_fake), logit_fake.numel(), carr, _p(content), _p(out), _p(dgen),
         pix_ld(dgen, C) if dgen is not None else C, _p(dlogit_real_d), _p(dlogit_fake_d), _p(dlogit_fake_g), _p(buf),
         n, _stream())
    return out
