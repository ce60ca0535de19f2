"""Layer-graph executor for the SRGAN / FastSRGAN / Autoencoder networks and
the frozen VGG19 feature extractor, on libdgan.

The reference builds these networks as Keras functional models and lets
GradientTape differentiate them (srgan.py:129-272, fsrgan.py:99-258,
autoencoder.py:89-229, train_*.py train_step).  Here a model is a small
static graph of fused layer nodes built once (`Graph`), and `GraphPlan`
turns it into a fixed forward + backward schedule for one input shape:

  * every node is one libdgan call (Conv2D with its bias and activation
    fused into the GEMM epilogue, BN with its activation fused into the
    apply pass, PReLU with depth_to_space fused, ...);
  * activations are NHWC fp32 buffers whose pixel stride is rounded up to a
    multiple of 4 floats (16-byte aligned rows for the vector paths);
  * channel concatenation (autoencoder.py:134-138) is zero-copy: the members
    are written straight into channel slices of the concat buffer and their
    gradients accumulate there in place;
  * a tensor with several consumers (residual skips) accumulates its
    gradient with beta = 1 after the first writer, decided at plan time;
  * trainable variables live in one flat arena (`nets.Arena`) laid out in
    backward-completion order, so Adam is one launch and DP buckets become
    final front to back.

Nothing here computes on the host: PyTorch only allocates device memory.
"""
import math
import os

import numpy as np
import torch

from . import ops
from .nets import Arena, BNState

# ---------------------------------------------------------------------------
# graph definition
# ---------------------------------------------------------------------------


class Tensor:
    __slots__ = ("id", "C", "node")

    def __init__(self, tid, C, node):
        self.id, self.C, self.node = tid, C, node

    def __repr__(self):
        return f"T{self.id}(C={self.C}, from={self.node.kind}:{self.node.name})"


class Node:
    __slots__ = ("kind", "name", "ins", "out", "attrs", "idx")

    def __init__(self, kind, name, ins, attrs, idx):
        self.kind, self.name, self.ins, self.attrs, self.idx = kind, name, list(ins), dict(attrs), idx
        self.out = None


class Graph:
    """A Keras-functional-style network description (NHWC, channels only;
    spatial sizes are resolved per input shape by GraphPlan)."""

    def __init__(self, name, in_ch=3):
        self.name = name
        self.nodes = []
        self.vars = []          # (name, shape, init) in creation (Keras trainable_variables) order
        self.bn_layers = {}     # name -> channels
        self._names = {}
        self.input = self._node("input", "input", [], in_ch)
        self.output = None

    def _uname(self, base):
        k = self._names.get(base, 0)
        self._names[base] = k + 1
        return base if k == 0 else f"{base}_{k}"

    def _node(self, kind, name, ins, C, **attrs):
        n = Node(kind, name, ins, attrs, len(self.nodes))
        n.out = Tensor(len(self.nodes), C, n)
        self.nodes.append(n)
        return n.out

    def _var(self, name, shape, init):
        self.vars.append((name, tuple(int(s) for s in shape), init))

    # layers ---------------------------------------------------------------
    def conv(self, x, filters, kernel, strides=1, padding="same", use_bias=True, act=None, alpha=0.3,
             kernel_init=("glorot_uniform",), name=None):
        """keras.layers.Conv2D (HWIO kernel), bias and activation fused."""
        name = self._uname(name or "conv2d")
        self._var(f"{name}/kernel", (kernel, kernel, x.C, filters), kernel_init)
        if use_bias:
            self._var(f"{name}/bias", (filters,), ("zeros",))
        return self._node("conv", name, [x], filters, k=kernel, s=strides, padding=padding, bias=use_bias,
                          act=act, alpha=alpha)

    def bn(self, x, momentum=0.99, epsilon=1e-3, act=None, alpha=0.3, gamma_init=("ones",), name=None):
        """keras.layers.BatchNormalization (+ the activation that follows it, fused)."""
        name = self._uname(name or "batch_normalization")
        self._var(f"{name}/gamma", (x.C,), gamma_init)
        self._var(f"{name}/beta", (x.C,), ("zeros",))
        self.bn_layers[name] = x.C
        return self._node("bn", name, [x], x.C, momentum=momentum, eps=epsilon, act=act, alpha=alpha)

    def prelu(self, x, block=1, name=None):
        """keras.layers.PReLU(shared_axes=[1, 2]), after tf.nn.depth_to_space(x, block) when block == 2."""
        if x.C % (block * block):
            raise ValueError("depth_to_space needs channels divisible by block^2")
        C = x.C // (block * block)
        name = self._uname(name or "p_re_lu")
        self._var(f"{name}/alpha", (1, 1, C), ("zeros",))
        return self._node("prelu", name, [x], C, block=block)

    def add(self, a, b, name=None):
        if a.C != b.C:
            raise ValueError("Add needs equal channels")
        return self._node("add", self._uname(name or "add"), [a, b], a.C)

    def concat(self, a, b, name=None):
        return self._node("concat", self._uname(name or "concatenate"), [a, b], a.C + b.C)

    def maxpool(self, x, name=None):
        return self._node("maxpool", self._uname(name or "max_pooling2d"), [x], x.C)

    def upsample_relu(self, x, name=None):
        return self._node("upsample", self._uname(name or "up_sampling2d"), [x], x.C)

    def dwconv(self, x, use_bias=True, kernel_init=("glorot_uniform",), name=None):
        """keras.layers.DepthwiseConv2D(3, strides 1, 'same')."""
        name = self._uname(name or "depthwise_conv2d")
        self._var(f"{name}/depthwise_kernel", (3, 3, x.C, 1), kernel_init)
        if use_bias:
            self._var(f"{name}/bias", (x.C,), ("zeros",))
        return self._node("dwconv", name, [x], x.C, bias=use_bias)

    def act(self, x, act, alpha=0.3, name=None):
        return self._node("act", self._uname(name or "activation"), [x], x.C, act=act, alpha=alpha)

    def set_output(self, t):
        self.output = t
        return self

    # derived ----------------------------------------------------------------
    def var_list(self):
        return [(n, s) for n, s, _ in self.vars]

    def layout_order(self):
        """Backward-completion order: variables of the last layer first."""
        return [n for n, _, _ in reversed(self.vars)]

    def consumers(self):
        out = {n.out.id: [] for n in self.nodes}
        for n in self.nodes:
            for t in n.ins:
                out[t.id].append(n)
        return out


# ---------------------------------------------------------------------------
# Keras-style initialisers from a seeded numpy PCG64 stream
# ---------------------------------------------------------------------------
def _fans(shape):
    if len(shape) == 4:
        rf = shape[0] * shape[1]
        return shape[2] * rf, shape[3] * rf
    if len(shape) == 2:
        return shape[0], shape[1]
    return int(np.prod(shape)), int(np.prod(shape))


def _trunc_normal(rng, shape, std):
    out = rng.standard_normal(shape)
    bad = np.abs(out) > 2.0
    while bad.any():
        out[bad] = rng.standard_normal(int(bad.sum()))
        bad = np.abs(out) > 2.0
    return out * std


def init_value(rng, shape, init):
    kind = init[0]
    if kind == "zeros":
        return np.zeros(shape, np.float32)
    if kind == "ones":
        return np.ones(shape, np.float32)
    if kind == "normal":  # tf.random_normal_initializer(mean, stddev)
        return (init[1] + init[2] * rng.standard_normal(shape)).astype(np.float32)
    fan_in, fan_out = _fans(shape)
    if kind == "glorot_uniform":
        lim = math.sqrt(6.0 / (fan_in + fan_out))
        return rng.uniform(-lim, lim, shape).astype(np.float32)
    if kind == "he_normal":  # VarianceScaling(2, fan_in, truncated_normal)
        return _trunc_normal(rng, shape, math.sqrt(2.0 / fan_in) / 0.87962566103423978).astype(np.float32)
    if kind == "lecun_normal":
        return _trunc_normal(rng, shape, math.sqrt(1.0 / fan_in) / 0.87962566103423978).astype(np.float32)
    if kind == "he_normal_plain":  # untruncated N(0, 2/fan_in): seeded stand-in for pretrained VGG weights
        return (rng.standard_normal(shape) * math.sqrt(2.0 / fan_in)).astype(np.float32)
    raise ValueError(f"unknown initialiser {init!r}")


def init_graph_variables(graph, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    return {n: init_value(rng, s, init) for n, s, init in graph.vars}


# ---------------------------------------------------------------------------
# static plan
# ---------------------------------------------------------------------------
def _ld(C):
    """Pixel stride of an activation buffer: channel counts >= 4 round up to a
    multiple of 4 floats (16-byte rows); narrow tensors (logits, images) stay dense."""
    return C if C < 4 else -(-C // 4) * 4


def _buf(N, H, W, C, device):
    """NHWC buffer with a 16-byte-multiple pixel stride; returns the [..., :C] view."""
    ld = _ld(C)
    t = torch.empty((N, H, W, ld), dtype=torch.float32, device=device)
    return t if ld == C else t[..., :C]


class GraphPlan:
    """Forward/backward schedule of a Graph for input [N, H, W, Cin].

    slots: independent activation sets (e.g. D(real) and D(fake), or VGG on
    G(x) and on the target) whose backwards run after all forwards.
    param_grads: False for frozen networks (VGG19) -- only input gradients.
    alias: a plan of the same graph over a larger batch whose slot-0
    activations this plan's slot 0 views (its first N images): e.g. a
    backward over one half of a batched forward."""

    def __init__(self, graph, N, H, W, arena, bn_state, device, slots=1, train=True, param_grads=True,
                 alias=None, math=None):
        self.g = graph
        self.arena, self.bn = arena, bn_state
        self.device = device
        self.N = N
        self.train = train
        self.param_grads = param_grads
        nodes = graph.nodes
        cons = graph.consumers()
        # ---- shape inference + descriptors ----
        shp = {}
        self.desc = {}
        shp[graph.input.id] = (N, H, W, graph.input.C)
        for n in nodes[1:]:
            x = shp[n.ins[0].id]
            _, h, w, c = x
            if n.kind == "conv":
                d = ops.ConvDesc(N, h, w, c, n.out.C, n.attrs["k"], n.attrs["s"], n.attrs["padding"], math=math)
                d.label = f"{graph.name}.{n.name}"
                self.desc[n.idx] = d
                shp[n.out.id] = d.out_shape
            elif n.kind == "prelu":
                b = n.attrs["block"]
                shp[n.out.id] = (N, h * b, w * b, n.out.C)
            elif n.kind == "maxpool":
                shp[n.out.id] = (N, h // 2, w // 2, c)
            elif n.kind == "upsample":
                shp[n.out.id] = (N, 2 * h, 2 * w, c)
            elif n.kind == "concat":
                y = shp[n.ins[1].id]
                if y[1:3] != x[1:3]:
                    raise ValueError(f"concat {n.name}: spatial mismatch {x} vs {y}")
                shp[n.out.id] = (N, h, w, n.out.C)
            elif n.kind == "add":
                y = shp[n.ins[1].id]
                if y != x:
                    raise ValueError(f"add {n.name}: shape mismatch {x} vs {y}")
                shp[n.out.id] = x
            else:  # bn, dwconv, act
                shp[n.out.id] = x
        self.shape = shp
        self.out_shape = shp[graph.output.id]
        # ---- zero-copy concat membership ----
        # member t of concat node c becomes a channel slice of c's buffer when t is
        # produced by a node (not the graph input), belongs to one concat only, and
        # every other consumer of t precedes c's consumers (their gradient
        # contributions then accumulate after c's consumer has written the slice).
        self.slice_of = {}   # tensor id -> (concat tensor id, channel offset)
        for n in nodes:
            if n.kind != "concat":
                continue
            off = 0
            first_cons = min((m.idx for m in cons[n.out.id]), default=len(nodes))
            for t in n.ins:
                ok = (t.id != graph.input.id and t.id not in self.slice_of and t.id != graph.output.id
                      and all(m.idx < first_cons for m in cons[t.id]))
                if ok:
                    self.slice_of[t.id] = (n.out.id, off)
                off += t.C
        # ---- fused activation gradients ----
        # a conv whose activation output feeds exactly one consumer that can fold
        # act'(z) into the gradient it writes (a conv's masked bwd_data epilogue, a
        # max-pool's routing pass, or -- for ReLU -- the nearest-upsample+ReLU
        # backward, whose x > 0 mask is the same) skips its own act_bwd pass.
        self.premask = set()
        for n in nodes[1:]:
            if n.kind != "conv" or ops.act_id(n.attrs["act"]) == 0 or n.out.id == graph.output.id:
                continue
            cs = cons[n.out.id]
            if len(cs) != 1 or n.out.id in self.slice_of:
                continue
            c = cs[0]
            if c.kind in ("conv", "maxpool") or (c.kind == "upsample" and ops.act_id(n.attrs["act"]) == 2):
                self.premask.add(n.out.id)
        # ---- BatchNorm + residual Add ----
        # a linear BN whose only consumer is an Add (the SR residual blocks, srgan.py:165 /
        # :180, fsrgan.py:176 / :214) writes act(BN(y)) + skip straight into the Add's output
        # in a training forward; backward, the BN reads the Add's output gradient (aliased:
        # the Add passes it through unchanged) and the Add only routes it to the skip input
        self.bn_add = {}   # bn node idx -> (add node, skip input tensor)
        for a in (nodes[1:] if train and not os.environ.get("DG_NO_BN_ADD") else []):
            if a.kind != "add" or a.out.id in self.slice_of or a.out.id == graph.output.id:
                continue
            for t, o in ((a.ins[0], a.ins[1]), (a.ins[1], a.ins[0])):
                b = t.node
                # the skip must be final when the BN runs: produced by an earlier node
                # (the graph input is node 0)
                if (b.kind == "bn" and ops.act_id(b.attrs["act"]) == 0 and len(cons[t.id]) == 1
                        and t.id not in self.slice_of and o.id != t.id and b.idx not in self.bn_add
                        and o.node.idx < b.idx):
                    self.bn_add[b.idx] = (a, o)
                    break
        self.add_of_bn = {a.idx: nodes[b] for b, (a, _) in self.bn_add.items()}   # add idx -> its BN
        # ---- activation buffers per slot ----
        self.slots = []
        for k in range(slots):
            if alias is not None and k == 0:
                self.slots.append({tid: t[:N] for tid, t in alias.slots[0].items() if tid != graph.input.id})
            else:
                self.slots.append(self._alloc_set(nodes, shp))
        self.saved = []
        for _ in range(slots):
            s = {}
            for n in nodes:
                if n.kind == "bn":
                    s[n.name] = (torch.empty(n.out.C, device=device), torch.empty(n.out.C, device=device))
            self.saved.append(s)
        # ---- gradient buffers (shared by slots) + beta schedule ----
        if train:
            self.grad = self._alloc_set(nodes, shp)
            self._schedule(nodes, cons)
            self._alias_add_grads(nodes, cons)
            mx = 0
            for n in nodes[1:]:
                if n.kind in ("conv", "bn", "act"):
                    s0 = shp[n.out.id]
                    mx = max(mx, int(np.prod(s0[:3])) * _ld(s0[3]))
            self.scratch = torch.empty(max(mx, 4), dtype=torch.float32, device=device)
        # ---- bf16x6 operand planes shared between the ops of a conv ----
        # w: one buffer per conv of the NETWORK and weight-plane layout
        # (arena.wplanes[(layer, format, bytes)]), shared by all its plans of that
        # layout (e.g. the VGG19 forward over 2N images and the backward over N);
        # plans whose GEMMs run another arithmetic (a VGG19 planned at 32^2 on
        # bf16x6 and at 256^2 on fp16x3) get buffers of their own, each stamped
        # with the weight version it was split from; x: per slot, split by fwd and
        # kept for bwd_filter (trainable plans that own their activations); dy: one
        # scratch per plan.
        wplanes = getattr(arena, "wplanes", None)
        if wplanes is None:
            wplanes = arena.wplanes = {}
        conv_nodes = [n for n in nodes[1:] if n.kind == "conv"]
        descs = [self.desc[n.idx] for n in conv_nodes]
        keep_x = train and param_grads and alias is None
        # fp16 weight copies of a trainable network: views into one fp16 shadow of the
        # arena (arena.half), converted by ONE launch per forward (dg_to_f16) instead of
        # one conversion per conv (the weights change with every Adam step)
        half = (not getattr(arena, "frozen", False) and not os.environ.get("DG_NO_F16_WARENA")
                and any(d.math == ops.MATH_FP16 and (d.plane_mask[0] | d.plane_mask[1]) & ops.TENSOR_W
                        for d in descs))
        if half and getattr(arena, "half", None) is None:
            arena.half = torch.empty(arena.numel, dtype=torch.float16, device=device)
        self.half_w = set()   # conv node idx whose fp16 weight copy is an arena.half view
        self.cplanes = []
        for k in range(slots):
            wb = []
            for n, d in zip(conv_nodes, descs):
                if (d.plane_mask[0] | d.plane_mask[1]) & ops.TENSOR_W:
                    h16 = half and d.math == ops.MATH_FP16
                    lay = ops.weight_layout(d)
                    key = (n.name, "f16") if h16 else (n.name,) + lay
                    if key not in wplanes:
                        if h16:
                            wname = f"{n.name}/kernel"
                            o, cnt = arena.offsets[wname], int(np.prod(arena.shapes[wname]))
                            assert 2 * cnt <= d.plane_bytes(ops.TENSOR_W)   # (sized for bf16x6 planes)
                            wplanes[key] = ops.PlaneBuf.over(arena.half[o:o + cnt].view(torch.uint8), lay)
                        else:
                            wplanes[key] = ops.PlaneBuf(lay[1], device, lay[0])
                    if h16:
                        self.half_w.add(n.idx)
                    wb.append(wplanes[key])
                else:
                    wb.append(None)
            ps = ops.plan_planes(descs, device, keep_x=keep_x, wbufs=wb)
            if not train:
                for p in ps:
                    p.dy = None
            if k > 0 and train:
                for p, p0 in zip(ps, self.cplanes[0].values()):
                    p.dy = p0.dy   # one dy scratch per plan
            self.cplanes.append({n.idx: p for n, p in zip(conv_nodes, ps)})
        # producer-written planes on conv -> conv chains (VGG19): a conv whose
        # activation output feeds exactly one conv (premask) writes that
        # consumer's x planes in its forward epilogue, and the consumer's
        # input-gradient epilogue writes the producer's dy planes -- no split
        # pass for either tensor.  Every fed tensor has a buffer of its own.
        self.fed_x, self.fed_dy = set(), set()
        self.pool_out = [dict() for _ in range(slots)]    # maxpool node -> consumer conv's x planes
        self.pool_gout = [dict() for _ in range(slots)]   # maxpool node -> producer conv's dy planes
        feed = not os.environ.get("DG_NO_FEED")
        # (producer-written planes are bf16x6 or, for a consumer whose forward runs fp16x3,
        # fp16x3 planes -- the PlaneBuf's fmt tells the producer; an fp16 descriptor's
        # planes are the fp16 copies its own ops convert, so neither end of a feed may be fp16)
        x6 = lambda d: d.math in (ops.MATH_BF16X6, ops.MATH_F16X3)   # noqa: E731
        for m in (nodes[1:] if feed else []):
            # max pool between two convs: its output is the next conv's input,
            # its input gradient the previous conv's dy (premask: act' folded in)
            if m.kind != "maxpool" or m.out.C % 16:
                continue
            cs = cons[m.out.id]
            if len(cs) == 1 and cs[0].kind == "conv" and m.out.id not in self.slice_of:
                c = cs[0]
                dc = self.desc[c.idx]
                if dc.plane_mask[ops.OP_FWD] & ops.TENSOR_X and x6(dc):
                    for k in range(slots):
                        pc = self.cplanes[k][c.idx]
                        if pc.x is None:
                            pc.x = ops.PlaneBuf(dc.plane_bytes(ops.TENSOR_X), device, dc.plane_format(ops.TENSOR_X))
                        self.pool_out[k][m.idx] = pc.x
                    self.fed_x.add(c.idx)
            t_in = m.ins[0]
            n = t_in.node
            if train and n.kind == "conv" and t_in.id in self.premask:
                dn = self.desc[n.idx]
                if (dn.plane_mask[ops.OP_BWD_DATA] | dn.plane_mask[ops.OP_BWD_FILTER]) & ops.TENSOR_DY and x6(dn):
                    for k in range(slots):
                        pn = self.cplanes[k][n.idx]
                        pn.dy = ops.PlaneBuf(dn.plane_bytes(ops.TENSOR_DY), device, dn.plane_format(ops.TENSOR_DY))
                        self.pool_gout[k][m.idx] = pn.dy
                    self.fed_dy.add(n.idx)
        for n in (conv_nodes if feed else []):
            t = n.out
            if t.id not in self.premask or cons[t.id][0].kind != "conv":
                continue
            c = cons[t.id][0]
            dn, dc = self.desc[n.idx], self.desc[c.idx]
            if dn.Cout % 16 or not (x6(dn) and x6(dc)):
                continue
            if dc.plane_mask[ops.OP_FWD] & ops.TENSOR_X:
                for k in range(slots):
                    pc = self.cplanes[k][c.idx]
                    if pc.x is None:
                        pc.x = ops.PlaneBuf(dc.plane_bytes(ops.TENSOR_X), device, dc.plane_format(ops.TENSOR_X))
                    self.cplanes[k][n.idx].fwd_out = pc.x
                self.fed_x.add(c.idx)
            if train and (dn.plane_mask[ops.OP_BWD_DATA] | dn.plane_mask[ops.OP_BWD_FILTER]) & ops.TENSOR_DY:
                for k in range(slots):
                    pn = self.cplanes[k][n.idx]
                    pn.dy = ops.PlaneBuf(dn.plane_bytes(ops.TENSOR_DY), device, dn.plane_format(ops.TENSOR_DY))
                    self.cplanes[k][c.idx].bwd_out = pn.dy
                self.fed_dy.add(n.idx)
        # ---- fp16 operand copies written by their producers (mixed_float16) ----
        # an fp16 conv reads fp16 copies of x and dy (its dg_conv_planes_t buffers, converted
        # per call otherwise): the BN / PReLU / Add producing its input writes the x copy beside
        # its fp32 output, and the BN / PReLU right after it, whose backward produces its output
        # gradient, writes the dy copy -- no conversion launch before the GEMMs
        self.h_x_out = {}    # producer node idx -> consuming conv node idx
        self.h_dy_out = {}   # node idx -> the conv node whose dy its backward writes
        f16 = lambda d: d.math == ops.MATH_FP16   # noqa: E731
        for c in (conv_nodes if (train and feed and not os.environ.get("DG_NO_F16_FEED")) else []):
            dc = self.desc[c.idx]
            if not f16(dc):
                continue
            t, p = c.ins[0], c.ins[0].node
            if (dc.plane_mask[ops.OP_FWD] & ops.TENSOR_X and p.kind in ("bn", "prelu", "add")
                    and t.id not in self.slice_of and p.idx not in self.h_x_out
                    and sum(1 for m in cons[t.id] if m.kind == "conv") == 1
                    and all(self.cplanes[k][c.idx].x is not None for k in range(slots))):
                self.h_x_out[p.idx] = c.idx
            cs = cons[c.out.id]
            if (len(cs) == 1 and cs[0].kind in ("bn", "prelu") and cs[0].idx == c.idx + 1
                    and ops.act_id(c.attrs["act"]) == 0 and c.out.id not in self.slice_of
                    and (dc.plane_mask[ops.OP_BWD_DATA] | dc.plane_mask[ops.OP_BWD_FILTER]) & ops.TENSOR_DY
                    and self.cplanes[0][c.idx].dy is not None):
                self.h_dy_out[cs[0].idx] = c.idx
        # ---- max pools fused into their conv's forward epilogue ----
        # a conv (ReLU / LeakyReLU / linear) whose output feeds only a 2x2 max
        # pool, on a plan that can run the pool in its epilogue, writes the
        # pooled values, their planes and a {argmax, sign} byte per pooled
        # element instead of its full-size activation; the pool's backward
        # routes from those bytes.  An aliasing plan follows its forward plan.
        self.fused_pool = {}   # maxpool node idx -> producing conv node
        self.pool_idx = [dict() for _ in range(slots)]
        if alias is not None:
            self.fused_pool = dict(alias.fused_pool)
        elif not os.environ.get("DG_NO_FUSED_POOL"):
            for m in nodes[1:]:
                if m.kind != "maxpool":
                    continue
                t_in = m.ins[0]
                n = t_in.node
                if (n.kind != "conv" or len(cons[t_in.id]) != 1 or t_in.id in self.slice_of
                        or t_in.id == graph.output.id or ops.act_id(n.attrs["act"]) not in (0, 1, 2)):
                    continue
                if self.desc[n.idx].pool_fusable(n.attrs["act"]):
                    self.fused_pool[m.idx] = n
        self.fused_conv = {n.idx: m for m, n in ((nodes[i], c) for i, c in self.fused_pool.items())}
        for k in range(slots):
            for midx in self.fused_pool:
                if alias is not None and k == 0:
                    self.pool_idx[k][midx] = alias.pool_idx[0][midx][:N]
                else:
                    self.pool_idx[k][midx] = torch.empty(shp[nodes[midx].out.id], dtype=torch.uint8, device=device)
        # ---- planes-only activations ----
        # in a plan without parameter gradients (the frozen VGG19), a conv whose
        # activation output feeds exactly one conv as producer-written planes
        # skips its fp32 output: the consumer's forward reads the planes, and its
        # masked input gradient takes act' from the planes' sign
        # (dg_conv_bwd_data_xmask).  An aliasing plan reads its forward plan's
        # planes (the first N images' rows).
        self.nofp32 = set()
        if alias is not None:
            self.nofp32 = set(alias.nofp32)
            for n in conv_nodes:
                if n.idx not in self.nofp32:
                    continue
                c = cons[n.out.id][0]
                src = alias.cplanes[0][c.idx].x
                self.cplanes[0][c.idx].x = src.view(self.desc[c.idx].plane_bytes(ops.TENSOR_X))
        elif not param_grads and feed and not os.environ.get("DG_NO_PLANES_ONLY"):
            for n in conv_nodes:
                t = n.out
                if (n.idx in self.fused_conv or t.id == graph.output.id or t.id not in self.premask
                        or ops.act_id(n.attrs["act"]) not in (0, 1, 2)):
                    continue
                c = cons[t.id][0]
                if c.kind == "conv" and all(self.cplanes[k][n.idx].fwd_out is not None for k in range(slots)):
                    self.nofp32.add(n.idx)
        # ---- fp16x3 input gradients (DG_MATH_F16X3: VGG19's backward) ----
        # a gradient has no static range: each fp16x3 dy is scaled from a bound of its max
        # (include/dgan.h dg_conv_set_grad_scale).  Per conv a device max slot gmax (max |dy|
        # of that conv, written by atomicMax by the op that produces it) and a weight bound
        # gwb (max_ci sum |w|, recomputed when the frozen weights change).  A conv's dy planes
        # written by its consumer conv c are scaled from (gmax[c], gwb[c]) (|dy| <= that
        # product); written by a pool's backward or split from the fp32 graph-output gradient,
        # from their measured max gmax[itself].
        self.x3_top = None
        self.x3_measure_dy = set()   # convs whose fp32 dy is measured (absmax) before their backward ops
        x3g = [n for n in conv_nodes if train and self.desc[n.idx].plane_format(ops.TENSOR_DY) == ops.PLANES_F16X3]
        if x3g:
            slot_of = {n.idx: i for i, n in enumerate(conv_nodes)}
            self._x3_slot = slot_of
            self.gmax = ops.max_slot(len(conv_nodes), device=device)
            self.gwb = torch.zeros(len(conv_nodes), dtype=torch.float32, device=device)
            self._gwb_ver = None
            self.x3_convs = [n for n in x3g]
            gm = lambda n: self.gmax[slot_of[n.idx]]                      # noqa: E731
            gw = lambda n: self.gwb[slot_of[n.idx]:slot_of[n.idx] + 1]    # noqa: E731
            self.pool_gscale = {}   # fused maxpool node idx -> scale source of the dy planes it writes

            def producer_conv(t):
                """The conv whose output is t, directly or through one 2x2 max pool."""
                nd = t.node
                if nd.kind == "maxpool":
                    nd = nd.ins[0].node
                return nd if nd.kind == "conv" else None

            for n in x3g:
                d = self.desc[n.idx]
                cs = cons[n.out.id]
                if n.out.id == graph.output.id:
                    src = (gm(n), None)   # the caller's fp32 gradient: max measured in backward()
                    self.x3_top = n
                elif len(cs) == 1 and cs[0].kind == "conv" and n.idx in self.fed_dy:
                    src = (gm(cs[0]), gw(cs[0]))
                elif len(cs) == 1 and cs[0].kind == "maxpool":
                    src = (gm(n), None)   # the pool's input gradient: max written by the pool's consumer
                    if cs[0].idx in self.fused_pool:
                        self.pool_gscale[cs[0].idx] = src
                    else:   # (an unfused pool's backward writes fp32 only; the conv splits it)
                        for k in range(slots):
                            self.pool_gout[k].pop(cs[0].idx, None)
                        self.fed_dy.discard(n.idx)
                else:
                    # a gradient arriving from a BN / PReLU / Add / concat (the SR family under
                    # DG_CONV_MATH=f16x3): its max is measured in backward() before the conv's ops
                    src = (gm(n), None)
                    self.x3_measure_dy.add(n.idx)
                p = producer_conv(n.ins[0])
                d.set_grad_scale(dy_m=src[0], dy_g=src[1], dx_m=gm(n), dx_g=gw(n),
                                 dx_max=gm(p) if p is not None else None)
        # ---- fp16x3 activation scales (include/dgan.h dg_conv_set_act_scale) ----
        # a conv's fp16x3 x planes carry the scale their producer wrote them with.  A conv that
        # writes its consumer's planes -- in its epilogue, its fused pool's, or through an unfused
        # pool -- scales them from its output bound: (max |its input|, measured) x (max over output
        # channels of sum |w|) + max |bias| (awb, per weight version), and measures max |its
        # output| (the consumer's input) in the same epilogue.  Every other fp16x3 x operand is
        # measured by the op that splits it (a plain max slot).  VGG19's activations (a
        # preprocessed image of +-128 onwards) thus keep 22 bits down to 2^-17 of each bound.
        # The measured maxima are per slot (amax[slot]): a slot's forward re-measures them, and its
        # kept x planes must be read back (bwd_filter) with the scale of the slot that wrote them --
        # D(real) and D(fake) of the SR discriminator are two slots of one plan whose inputs may
        # sit in different binades.  The descriptors are shared by the slots, so each slot's scale
        # context is set on them before that slot's forward and backward (_use_act_slot; host-side
        # pointers, baked into the launches).
        self.act_feeds = {}      # producer conv idx -> (consumer conv node, unfused pool node or None)
        self.act_measure = []    # convs whose input max is measured before them (input not a conv's output)
        self.pool_scale = [dict() for _ in range(slots)]   # unfused maxpool idx -> its planes' scale source
        self.amax = self.awb = None
        self._awb_ver = None
        self._act_ctx = None     # per slot: [(desc, x source, y source, y_max)]
        self._act_slot = None
        if alias is None and any(self.desc[n.idx].plane_format(ops.TENSOR_X) == ops.PLANES_F16X3 for n in conv_nodes):
            ci = {n.idx: i for i, n in enumerate(conv_nodes)}
            self.amax = ops.max_slot(slots, len(conv_nodes), device=device)
            self.awb = torch.zeros(len(conv_nodes), 2, dtype=torch.float32, device=device)
            feeds = {}   # producer conv idx -> (consumer conv, unfused pool or None, planes it writes or None)
            for n in conv_nodes:
                cs = cons[n.out.id]
                if len(cs) != 1:
                    continue
                m, buf = None, None
                if cs[0].kind == "conv":
                    c, buf = cs[0], self.cplanes[0][n.idx].fwd_out
                elif cs[0].kind == "maxpool" and len(cons[cs[0].out.id]) == 1 and cons[cs[0].out.id][0].kind == "conv":
                    m, c = cs[0], cons[cs[0].out.id][0]
                    buf = self.pool_out[0].get(m.idx)
                else:
                    continue
                feeds[n.idx] = (c, m if (m is not None and n.idx not in self.fused_conv) else None, buf)
            self.act_feeds = {i: (c, m) for i, (c, m, buf) in feeds.items()
                              if buf is not None and buf.fmt == ops.PLANES_F16X3}
            producer = {c.idx: i for i, (c, _, _) in feeds.items()}

            def ysrc(n, k):
                i = ci[n.idx]
                return (self.amax[k, i], self.awb[i, 0:1], self.awb[i, 1:2] if n.attrs["bias"] else None)

            for i in self.act_feeds:
                # the producer's output bound needs max |its input|: measured by the epilogue of the
                # conv producing that input (any arithmetic), else by an absmax pass before it
                if i not in producer:
                    self.act_measure.append(i)
            self._act_ctx = []
            for k in range(slots):
                ctx = {n.idx: [None, None, None] for n in conv_nodes}   # x source, y source, y_max
                for i, (c, m) in self.act_feeds.items():
                    n = nodes[i]
                    ctx[i][1] = ysrc(n, k)
                    if m is not None:
                        self.pool_scale[k][m.idx] = ysrc(n, k)
                    if i in producer:
                        ctx[producer[i]][2] = self.amax[k, ci[i]]
                for n in conv_nodes:
                    if self.desc[n.idx].plane_format(ops.TENSOR_X) != ops.PLANES_F16X3:
                        continue
                    p = producer.get(n.idx)
                    ctx[n.idx][0] = ysrc(nodes[p], k) if p in self.act_feeds else (self.amax[k, ci[n.idx]],)
                self._act_ctx.append([(self.desc[i], x, y, ymax) for i, (x, y, ymax) in ctx.items()
                                      if x is not None or y is not None or ymax is not None])
            self._act_ci = ci
            self._use_act_slot(0)
        # ---- workspace ----
        ws = [0]
        for n in nodes[1:]:
            sx = shp[n.ins[0].id]
            if n.kind == "conv":
                ws.append(self.desc[n.idx].max_ws())
            elif n.kind == "bn":
                ws.append(ops.bn_workspace_bytes(int(np.prod(sx[:3])), sx[3]))
            elif n.kind == "prelu":
                b = n.attrs["block"]
                ws.append(ops.prelu_workspace_bytes(sx[0], sx[1], sx[2], n.out.C, b))
            elif n.kind == "dwconv":
                ws.append(ops.dwconv3_workspace_bytes(*sx))
        self.ws_bytes = max(ws)

    def _use_act_slot(self, slot):
        """Point the shared descriptors' fp16x3 activation scale context at slot's sources."""
        if self._act_ctx is None or self._act_slot == slot:
            return
        for d, x, y, ymax in self._act_ctx[slot]:
            d.set_act_scale(x=x, y=y, y_max=ymax)
        self._act_slot = slot

    def _alloc_set(self, nodes, shp):
        """tensor id -> NHWC view (graph input excluded: supplied per call)."""
        bufs = {}
        for n in nodes[1:]:
            if n.out.id in self.slice_of:
                continue
            bufs[n.out.id] = _buf(*shp[n.out.id], self.device)
        for tid, (cid, off) in self.slice_of.items():
            C = shp[tid][3]
            bufs[tid] = bufs[cid][..., off:off + C]
        return bufs

    def _alias_add_grads(self, nodes, cons):
        """An Add passes its output gradient unchanged to both inputs: an input whose
        gradient buffer can BE the Add's (no copy) shares it.  That is the fused BN's output
        (bn_add), and a skip input the Add writes first in backward order (beta 0) whose other
        consumers all run after every reader of the Add's gradient -- they then accumulate
        (beta 1) into the shared buffer after the BN / Add backward has read it.  Down the
        SR residual trunk (srgan.py:165-181) every block's input gradient thus lives in one
        buffer that each block's first conv accumulates into."""
        self.add_alias = {}   # add node idx -> ids of the inputs whose gradient is the Add's
        gin, gout = self.g.input.id, self.g.output.id
        shared = set()
        for a in (reversed(nodes[1:]) if not os.environ.get("DG_NO_ADD_ALIAS") else ()):
            if a.kind != "add" or a.out.id == gout:
                continue
            root = self.grad[a.out.id]
            al = set()
            bn = self.add_of_bn.get(a.idx)
            if bn is not None:   # (read by the BN's backward, at its place in the order)
                self.grad[bn.out.id] = root
                al.add(bn.out.id)
            lim = a.idx if bn is None else bn.idx
            for o in a.ins:
                if (o.id in al or o.id in (gin, gout) or o.id in self.slice_of or o.id in shared
                        or a.ins[0].id == a.ins[1].id or self.beta[(a.idx, o.id)] != 0.0
                        or not all(c.idx < lim for c in cons[o.id] if c is not a)):
                    continue
                self.grad[o.id] = root
                al.add(o.id)
                shared.add(o.id)
                break
            self.add_alias[a.idx] = al

    def _schedule(self, nodes, cons):
        """beta (0 = first writer, 1 = accumulate) of every input-gradient write, in backward order."""
        written = set()
        self.beta = {}
        gin = self.g.input.id

        def mark(tid):
            b = 1.0 if tid in written else 0.0
            written.add(tid)
            return b

        for n in reversed(nodes[1:]):
            if n.kind == "concat":
                # the concat buffer's gradient (written by its consumer) is the members' gradient
                for t in n.ins:
                    if t.id in self.slice_of and self.slice_of[t.id][0] == n.out.id:
                        if t.id in written:
                            raise RuntimeError(f"concat {n.name}: member gradient written before the concat's")
                        written.add(t.id)
                    else:
                        self.beta[(n.idx, t.id)] = mark(t.id)
                continue
            for t in n.ins:
                self.beta[(n.idx, t.id)] = mark(t.id)
        self.input_first_beta = None  # graph input: the caller's beta applies to its first write
        self._in_writes = [k for k in self.beta if k[1] == gin]

    # ---------------------------------------------------------------- forward
    def forward(self, x, slot=0, training=True, out=None, ws=None):
        """x: NHWC device view [N,H,W,Cin]; returns the output view (or writes into `out`)."""
        g = self.g
        A = self.arena
        s = self.slots[slot]
        s[g.input.id] = x
        # weight planes: re-split every forward, except for a frozen network
        # (VGG19 content loss) whose buffer holds the planes of the current weights
        frozen = getattr(A, "frozen", False)
        if self.amax is not None:
            self._use_act_slot(slot)
        if self.act_feeds:
            # fp16x3 activation scales: the output bounds' weight terms (frozen weights: once per
            # version) and this pass's measured maxima
            if not frozen or self._awb_ver != A.version:
                for i in self.act_feeds:
                    n = g.nodes[i]
                    j = self._act_ci[i]
                    ops.weight_bound(A.param(f"{n.name}/kernel"), self.awb[j, 0:1],
                                     bias=A.param(f"{n.name}/bias") if n.attrs["bias"] else None,
                                     c_out=self.awb[j, 1:2])
                self._awb_ver = A.version
            ops.fill(self.amax[slot], 0.0)
        if self.half_w:
            # every fp16 conv's weight copy of this network in one launch
            ops.to_f16(A.data, A.half)
        if out is not None:
            s[g.output.id] = out
        fed_now = set()   # convs whose fp16 x copy a producer wrote in this pass
        add_done = set()  # Adds their BN wrote in this pass

        def x_copy(n):
            c = self.h_x_out.get(n.idx)
            return None if c is None else self.cplanes[slot][c].x

        def x_copied(n):
            c = self.h_x_out.get(n.idx)
            if c is not None:
                self.cplanes[slot][c].x.ready = True
                fed_now.add(c)

        for n in g.nodes[1:]:
            xin = s[n.ins[0].id]
            y = s[n.out.id]
            k = n.kind
            if k == "conv":
                d = self.desc[n.idx]
                bias = A.param(f"{n.name}/bias") if n.attrs["bias"] else None
                P = self.cplanes[slot][n.idx]
                # (a fed input's planes were written by its producer in this pass)
                fed = n.idx in self.fed_x or n.idx in fed_now
                if n.idx in self.half_w:
                    P.invalidate(0 if fed else ops.TENSOR_X)
                    P.w.ready = True
                else:
                    P.invalidate((self._stale_w(P, frozen)) | (0 if fed else ops.TENSOR_X))
                if n.idx in self.act_measure:
                    ops.absmax(xin, self.amax[slot, self._act_ci[n.idx]])   # (zeroed above)
                mp = self.fused_conv.get(n.idx)
                if mp is not None:
                    d.fwd_pool(xin, A.param(f"{n.name}/kernel"), self.pool_idx[slot][mp.idx], bias=bias,
                               act=n.attrs["act"], alpha=n.attrs["alpha"], pool_y=s[mp.out.id], ws=ws, planes=P,
                               pool_planes=self.pool_out[slot].get(mp.idx))
                else:
                    d.fwd(xin, A.param(f"{n.name}/kernel"), None if n.idx in self.nofp32 else y, bias=bias,
                          act=n.attrs["act"], alpha=n.attrs["alpha"], ws=ws, planes=P)
            elif k == "bn":
                mean, inv = self.saved[slot][n.name]
                if training:
                    fa = self.bn_add.get(n.idx)
                    w = n if fa is None else fa[0]   # (the node whose output this call writes)
                    ops.bn_fwd_train(xin, A.param(f"{n.name}/gamma"), A.param(f"{n.name}/beta"), mean, inv,
                                     self.bn.mean[n.name], self.bn.var[n.name], s[w.out.id], act=n.attrs["act"],
                                     alpha=n.attrs["alpha"], momentum=n.attrs["momentum"], eps=n.attrs["eps"],
                                     ws=ws, f16_out=x_copy(w), res=None if fa is None else s[fa[1].id])
                    x_copied(w)
                    if fa is not None:
                        add_done.add(w.idx)
                else:
                    ops.bn_fwd_infer(xin, A.param(f"{n.name}/gamma"), A.param(f"{n.name}/beta"),
                                     self.bn.mean[n.name], self.bn.var[n.name], y, act=n.attrs["act"],
                                     alpha=n.attrs["alpha"], eps=n.attrs["eps"])
            elif k == "prelu":
                ops.prelu_fwd(xin, A.param(f"{n.name}/alpha"), y, block=n.attrs["block"], f16_out=x_copy(n))
                x_copied(n)
            elif k == "add":
                if n.idx not in add_done:
                    ops.add(xin, s[n.ins[1].id], y, f16_out=x_copy(n))
                    x_copied(n)
            elif k == "concat":
                off = 0
                for t in n.ins:
                    if self.slice_of.get(t.id, (None,))[0] != n.out.id:
                        ops.strided_copy(s[t.id], y[..., off:off + t.C])
                    off += t.C
            elif k == "maxpool":
                if n.idx not in self.fused_pool:   # (else done by its conv's epilogue)
                    ops.maxpool2_fwd(xin, y, planes_out=self.pool_out[slot].get(n.idx),
                                     scale=self.pool_scale[slot].get(n.idx))
            elif k == "upsample":
                ops.upsample2_relu_fwd(xin, y)
            elif k == "dwconv":
                bias = A.param(f"{n.name}/bias") if n.attrs["bias"] else None
                ops.dwconv3_fwd(xin, A.param(f"{n.name}/depthwise_kernel"), y, bias=bias)
            elif k == "act":
                ops.act_fwd(xin, y, n.attrs["act"], n.attrs["alpha"])
            else:
                raise ValueError(k)
        return s[g.output.id]

    def _stale_w(self, P, frozen):
        """TENSOR_W when P's weight planes must be split again before use, else 0: always for a
        trainable network (its weights change with every Adam step), for a frozen one when the
        buffer was split from another weight version.  The buffer is stamped with the current
        version (the op about to read it splits it when it is not ready)."""
        w = P.w
        if w is None:
            return 0
        if not frozen:
            return ops.TENSOR_W
        v = self.arena.version
        if w.stamp == v:
            return 0
        w.stamp = v
        return ops.TENSOR_W

    # --------------------------------------------------------------- backward
    def _update_weight_bounds(self):
        """gwb[conv] = max over input channels of sum |w| over taps and output channels
        (a bound of |dx| / max |dy| of the layer's input gradient; dg_weight_bound_in)."""
        for i, n in enumerate(m for m in self.g.nodes if m.kind == "conv"):
            ops.weight_bound_in(self.arena.param(f"{n.name}/kernel"), self.gwb[i:i + 1])   # HWIO

    def _scratch(self, shape):
        N, H, W, C = shape
        ld = _ld(C)
        v = self.scratch[:N * H * W * ld].view(N, H, W, ld)
        return v if ld == C else v[..., :C]

    def backward(self, dout, slot=0, param_beta=0.0, input_grad=None, input_beta=0.0, ws=None, on_grads_ready=None,
                 params=None):
        """dout: gradient of the graph output.  Parameter gradients go to the
        arena grad buffer (g = new + param_beta*g) unless param_grads (or the
        per-call `params`) is off; input_grad (NHWC view) receives dL/d(input)
        (+ input_beta*old)."""
        g = self.g
        A = self.arena
        s = self.slots[slot]
        gr = dict(self.grad)
        gr[g.output.id] = dout
        if self.amax is not None:
            self._use_act_slot(slot)   # (the kept x planes of this slot: its scale sources)
        if getattr(self, "x3_convs", None):
            # fp16x3 input gradients: weight bounds (frozen weights: once per version), the
            # per-step max slots, and the measured max of the gradient entering the graph
            if not getattr(A, "frozen", False) or self._gwb_ver != A.version:   # (trainable: every step)
                self._update_weight_bounds()
                self._gwb_ver = A.version
            ops.fill(self.gmax, 0.0)
            if self.x3_top is not None:
                i = [n.idx for n in g.nodes if n.kind == "conv"].index(self.x3_top.idx)
                ops.absmax(dout, self.gmax[i])
        gin = g.input.id
        if input_grad is not None:
            gr[gin] = input_grad
        pg = self.param_grads if params is None else bool(params)
        frozen = getattr(A, "frozen", False)
        in_seen = [False]

        def beta_of(n, t):
            if t.id == gin:
                if in_seen[0]:
                    return 1.0
                in_seen[0] = True
                return input_beta
            return self.beta[(n.idx, t.id)]

        def need(t):
            return t.id != gin or input_grad is not None

        fed_dy_now = set()   # convs whose fp16 dy copy the node after them wrote just now

        def dy_copy(n, b):
            c = self.h_dy_out.get(n.idx)
            return None if (c is None or b != 0.0) else self.cplanes[slot][c].dy

        def dy_copied(n, buf):
            if buf is not None:
                buf.ready = True
                fed_dy_now.add(self.h_dy_out[n.idx])

        for n in reversed(g.nodes[1:]):
            k = n.kind
            t_in = n.ins[0]
            dz = gr[n.out.id]
            if k == "conv":
                d = self.desc[n.idx]
                act = n.attrs["act"]
                if ops.act_id(act) != 0 and n.out.id not in self.premask:
                    dy = self._scratch(self.shape[n.out.id])
                    ops.act_bwd(dz, s[n.out.id], dy, act, n.attrs["alpha"])
                else:
                    dy = dz   # (already multiplied by act'(z) by the consumer when premasked)
                P = self.cplanes[slot][n.idx]
                # (else written just now: by the consumer's bwd_data, or as the fp16 copy)
                if n.idx not in self.fed_dy and n.idx not in fed_dy_now:
                    P.invalidate(ops.TENSOR_DY)
                if frozen:
                    # (a backward-only plan -- VGG19's N-image backward over its 2N forward -- may
                    # hold weight planes of a layout the forward plan does not share)
                    P.invalidate(self._stale_w(P, True))
                if n.idx in self.x3_measure_dy:
                    ops.absmax(dy, self.gmax[self._x3_slot[n.idx]])   # (gmax zeroed above)
                if pg:
                    db = A.grad_of(f"{n.name}/bias") if n.attrs["bias"] else None
                    d.bwd_filter(s[t_in.id], dy, A.grad_of(f"{n.name}/kernel"), dbias=db, beta=param_beta, ws=ws,
                                 planes=P)
                if need(t_in):
                    if t_in.node.idx in self.nofp32:
                        # (x exists as the planes its producer wrote in the forward)
                        pa = t_in.node.attrs
                        P.x.ready = True
                        d.bwd_data_xmask(dy, A.param(f"{n.name}/kernel"), gr[t_in.id], pa["act"], pa["alpha"],
                                         beta=beta_of(n, t_in), ws=ws, planes=P)
                    elif t_in.id in self.premask:
                        pa = t_in.node.attrs
                        d.bwd_data_masked(dy, A.param(f"{n.name}/kernel"), gr[t_in.id], s[t_in.id], pa["act"],
                                          pa["alpha"], beta=beta_of(n, t_in), ws=ws, planes=P)
                    else:
                        d.bwd_data(dy, A.param(f"{n.name}/kernel"), gr[t_in.id], beta=beta_of(n, t_in), ws=ws,
                                   planes=P)
            elif k == "bn":
                mean, inv = self.saved[slot][n.name]
                # a BN fused with its residual Add never wrote s[n.out.id]: only a linear BN
                # may be fused, whose backward does not read z (ops.bn_bwd passes NULL)
                assert n.idx not in self.bn_add or ops.act_id(n.attrs["act"]) == 0
                b = beta_of(n, t_in)
                tgt = gr[t_in.id] if b == 0.0 else self._scratch(self.shape[t_in.id])
                hc = dy_copy(n, b)
                ops.bn_bwd(dz, s[n.out.id], s[t_in.id], A.param(f"{n.name}/gamma"), mean, inv, tgt,
                           A.grad_of(f"{n.name}/gamma") if pg else None, A.grad_of(f"{n.name}/beta") if pg else None,
                           act=n.attrs["act"], alpha=n.attrs["alpha"], beta=param_beta, ws=ws, f16_out=hc)
                dy_copied(n, hc)
                if b != 0.0:
                    ops.accumulate(tgt, gr[t_in.id], b)
            elif k == "prelu":
                b = beta_of(n, t_in)
                hc = dy_copy(n, b)
                ops.prelu_bwd(s[t_in.id], A.param(f"{n.name}/alpha"), dz, gr[t_in.id],
                              dalpha=A.grad_of(f"{n.name}/alpha") if pg else None, block=n.attrs["block"],
                              beta=b, alpha_beta=param_beta, ws=ws, f16_out=hc)
                dy_copied(n, hc)
            elif k == "add":
                for t in n.ins:
                    # (a fused BN's or a skip input's gradient may BE this one: _alias_add_grads)
                    if need(t) and t.id not in self.add_alias.get(n.idx, ()):
                        ops.accumulate(dz, gr[t.id], beta_of(n, t))
            elif k == "concat":
                off = 0
                for t in n.ins:
                    if self.slice_of.get(t.id, (None,))[0] != n.out.id and need(t):
                        ops.accumulate(dz[..., off:off + t.C], gr[t.id], beta_of(n, t))
                    off += t.C
            elif k == "maxpool" and n.idx in self.fused_pool:
                if need(t_in):
                    pa = t_in.node.attrs
                    b = beta_of(n, t_in)
                    gout = self.pool_gout[slot].get(n.idx)
                    # the fp32 gradient is read only by a bias / filter gradient or an
                    # accumulation; the conv's input gradient reads its dy planes
                    keep = gout is None or pg or b != 0.0
                    _, H, W, C = self.shape[t_in.id]
                    ops.maxpool2_bwd_idx(self.pool_idx[slot][n.idx], dz, gr[t_in.id] if keep else None, C, H, W,
                                         beta=b, act=pa["act"] if t_in.id in self.premask else "none",
                                         alpha=pa["alpha"], planes_out=gout,
                                         scale=getattr(self, "pool_gscale", {}).get(n.idx))
            elif k == "maxpool":
                if need(t_in):
                    pa = t_in.node.attrs if t_in.id in self.premask else {"act": "none", "alpha": 0.0}
                    ops.maxpool2_bwd(s[t_in.id], dz, gr[t_in.id], beta=beta_of(n, t_in), act=pa["act"],
                                     alpha=pa["alpha"], planes_out=self.pool_gout[slot].get(n.idx))
            elif k == "upsample":
                if need(t_in):
                    ops.upsample2_relu_bwd(s[t_in.id], dz, gr[t_in.id], beta=beta_of(n, t_in))
            elif k == "dwconv":
                if pg:
                    db = A.grad_of(f"{n.name}/bias") if n.attrs["bias"] else None
                    ops.dwconv3_bwd_filter(s[t_in.id], dz, A.grad_of(f"{n.name}/depthwise_kernel"), dbias=db,
                                           beta=param_beta, ws=ws)
                if need(t_in):
                    ops.dwconv3_bwd_data(dz, A.param(f"{n.name}/depthwise_kernel"), gr[t_in.id],
                                         beta=beta_of(n, t_in))
            elif k == "act":
                if need(t_in):
                    b = beta_of(n, t_in)
                    tgt = gr[t_in.id] if b == 0.0 else self._scratch(self.shape[t_in.id])
                    ops.act_bwd(dz, s[n.out.id], tgt, n.attrs["act"], n.attrs["alpha"])
                    if b != 0.0:
                        ops.accumulate(tgt, gr[t_in.id], b)
            if pg and on_grads_ready is not None and k in ("conv", "bn", "prelu", "dwconv"):
                on_grads_ready(n.name)


# ---------------------------------------------------------------------------
# Keras-shaped network object over a Graph
# ---------------------------------------------------------------------------
class GraphNetwork:
    """What the reference's drivers touch on a tf.keras.Model: call,
    trainable_variables, count_params, summary, save / load_weights,
    get_weights / set_weights."""

    def __init__(self, graph, seed=1234, device=None, kind=None, trainable=True):
        from .models import default_device
        self.graph = graph
        self.name = graph.name
        self.kind = kind or graph.name
        self.device = device or default_device()
        self.arena = Arena(graph.var_list(), self.device, graph.layout_order())
        self.bn = BNState(dict(graph.bn_layers), self.device)
        self.arena.load(init_graph_variables(graph, seed))
        self.trainable = trainable
        # a frozen network's weights change only through arena.load (version
        # bump): its bf16x6 weight planes stay valid across forwards
        self.arena.frozen = not trainable
        # conv arithmetic of this network's plans (None: the library default,
        # "fp16": the reference's mixed_float16 policy, include/dgan.h DG_MATH_FP16)
        self.conv_math = None
        self._plans = {}

    @property
    def trainable_variables(self):
        if not self.trainable:
            return []
        return [self.arena.param(n) for n, _ in self.arena.var_list]

    @property
    def non_trainable_variables(self):
        out = [] if self.trainable else [self.arena.param(n) for n, _ in self.arena.var_list]
        for k in self.bn.mean:
            out += [self.bn.mean[k], self.bn.var[k]]
        return out

    @property
    def variables(self):
        return self.trainable_variables + self.non_trainable_variables

    def count_params(self):
        return self.arena.count + sum(int(t.numel()) for k in self.bn.mean for t in (self.bn.mean[k], self.bn.var[k]))

    def summary(self, print_fn=print):
        print_fn(f'Model: "{self.name}"')
        for n, s in self.arena.var_list:
            print_fn(f"  {n:<40s} {str(tuple(s)):<22s} {int(np.prod(s)):>12,d}")
        print_fn(f"Total params: {self.count_params():,d}")
        print_fn(f"Trainable params: {self.arena.count if self.trainable else 0:,d}")

    def plan(self, N, H, W, slots=1, train=False, param_grads=True, alias=None, tag=None):
        """tag: a distinct plan (own buffers) of the same shape -- e.g. two forwards that run
        concurrently on two streams."""
        key = (N, H, W, slots, train, param_grads, id(alias) if alias is not None else None, self.conv_math, tag)
        if key not in self._plans:
            self._plans[key] = GraphPlan(self.graph, N, H, W, self.arena, self.bn, self.device, slots=slots,
                                         train=train, param_grads=param_grads, alias=alias, math=self.conv_math)
        return self._plans[key]

    def __call__(self, x, training=False):
        from .models import to_device
        x = to_device(x, self.device)
        N, H, W, _ = x.shape
        p = self.plan(N, H, W)
        ws = ops.Workspace(self.device)
        ws.get(p.ws_bytes)
        y = p.forward(x, slot=0, training=training, ws=ws)
        return y.contiguous().clone()

    # weights -------------------------------------------------------------
    def state_dict(self):
        d = dict(self.arena.export())
        d.update(self.bn.export())
        return d

    def load_state_dict(self, d):
        self.arena.load({n: d[n] for n, _ in self.arena.var_list if n in d})
        self.bn.load(d)

    def get_weights(self):
        w = self.arena.export()
        bn = self.bn.export()
        return [w[n] for n, _ in self.arena.var_list] + [bn[k] for k in sorted(bn)]

    def set_weights(self, weights):
        names = [n for n, _ in self.arena.var_list]
        self.arena.load(dict(zip(names, weights[:len(names)])))
        bnk = sorted(self.bn.export())
        self.bn.load(dict(zip(bnk, weights[len(names):])))

    def save(self, path):
        import json
        import os
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        base = path[:-4] if path.endswith(".npz") else path
        np.savez(base + ".npz", **self.state_dict())
        with open(base + ".json", "w") as f:
            json.dump({"model": self.kind, "name": self.name}, f)

    def load_weights(self, path):
        p = path if path.endswith(".npz") else path + ".npz"
        with np.load(p, allow_pickle=False) as z:
            self.load_state_dict({k: z[k] for k in z.files})
