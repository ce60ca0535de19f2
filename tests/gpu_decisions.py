"""Read the HIP path's activation decisions back from its activation buffers
(test helper for mask-conditioned parity, see oracle/decisions.py).

Every decision is recovered from what the HIP kernels themselves stored:
  * ReLU / LeakyReLU (conv epilogue, BN apply, nearest-upsample + ReLU):
    the post-activation value z is > 0 exactly where the kernel took the
    positive branch (z = x for x > 0, 0 or alpha*x <= 0 otherwise);
  * PReLU: the sign of its stored input (alpha may have either sign);
  * 2x2 max pool: the first maximum of each window of the stored fp32 input,
    the element the backward kernel routes the gradient to.
Masks are returned on the host as numpy arrays keyed by the layer name the
oracle uses for the same site.
"""
import numpy as np
import torch

RELU_ACTS = ("relu", "lrelu", "leaky_relu")


def _pos(t):
    return (t.detach() > 0).cpu().numpy()


def pool_argmax(x):
    """First-maximum index (row-major 2x2 window) of every pool window of NHWC x."""
    N, H, W, C = x.shape
    x = x.detach()[:, :H // 2 * 2, :W // 2 * 2].float()
    win = x.reshape(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(N, H // 2, W // 2, C, 4)
    return win.cpu().argmax(dim=-1).numpy()


def _depth_to_space(m, b):
    N, H, W, CB = m.shape
    C = CB // (b * b)
    return m.reshape(N, H, W, b, b, C).transpose(0, 1, 3, 2, 4, 5).reshape(N, H * b, W * b, C)


def fused_pool_decisions(idx):
    """A pool fused into its conv's epilogue stores one byte per pooled element
    (bits 0-1 the argmax, bit 2 the activation's sign there): -> (argmax [N,H/2,W/2,C],
    (conv mask, known) at full size -- the conv's decision is known where the
    pool routes the gradient)."""
    b = idx.detach().cpu().numpy().astype(np.int64)
    arg = b & 3
    pos = (b & 4) != 0
    N, H2, W2, C = b.shape
    mask = np.zeros((N, H2, 2, W2, 2, C), dtype=bool)
    known = np.zeros_like(mask)
    for q in range(4):
        sel = arg == q
        known[:, :, q // 2, :, q % 2, :] = sel
        mask[:, :, q // 2, :, q % 2, :] = sel & pos
    return arg, (mask.reshape(N, 2 * H2, 2 * W2, C), known.reshape(N, 2 * H2, 2 * W2, C))


def plane_positive(pbuf, shape):
    """x > 0 from the hi plane of a packed plane buffer for an NHWC shape: bf16x6
    [pixel][C/16][3][16] or fp16x3 [pixel][C/32][2][32] (pbuf.fmt); a positive bf16 /
    fp16 is a positive int16."""
    from dgan import ops
    N, H, W, C = shape
    if getattr(pbuf, "fmt", ops.PLANES_BF16X6) == ops.PLANES_F16X3:
        hi = pbuf.buf[:N * H * W * C * 4].view(torch.int16).reshape(N * H * W, C // 32, 2, 32)[:, :, 0, :]
    else:
        hi = pbuf.buf[:N * H * W * C * 6].view(torch.int16).reshape(N * H * W, C // 16, 3, 16)[:, :, 0, :]
    return (hi.reshape(N, H, W, C) > 0)


def graph_decisions(plan, slot=0, rows=None):
    """{layer name: mask / argmax} of one dgan.graph.GraphPlan slot; rows: a
    slice of the batch (e.g. one half of a batched forward)."""
    g = plan.g
    s = plan.slots[slot]
    sel = (lambda t: t) if rows is None else (lambda t: t[rows])
    out = {}
    fused_conv = getattr(plan, "fused_conv", {})
    nofp32 = getattr(plan, "nofp32", set())
    cons = g.consumers() if nofp32 else {}
    for n in g.nodes[1:]:
        k = n.kind
        if k == "conv" and n.idx in nofp32:
            # planes-only activation: the sign of the planes its consumer reads
            c = cons[n.out.id][0]
            out[n.name] = sel(plane_positive(plan.cplanes[slot][c.idx].x, plan.shape[n.out.id])).cpu().numpy()
        elif k == "conv" and n.idx in fused_conv:
            m = fused_conv[n.idx]
            arg, cm = fused_pool_decisions(sel(plan.pool_idx[slot][m.idx]))
            out[m.name] = arg
            if n.attrs.get("act") in RELU_ACTS:
                out[n.name] = cm
        elif k == "maxpool" and n.idx in getattr(plan, "fused_pool", {}):
            continue
        elif k in ("conv", "bn", "act") and n.attrs.get("act") in RELU_ACTS:
            out[n.name] = _pos(sel(s[n.out.id]))
        elif k == "upsample":
            out[n.name] = _pos(sel(s[n.out.id]))
        elif k == "prelu":
            m = _pos(sel(s[n.ins[0].id]))
            b = n.attrs["block"]
            out[n.name] = _depth_to_space(m, b) if b > 1 else m
        elif k == "maxpool":
            out[n.name] = pool_argmax(sel(s[n.ins[0].id]))
    return out


def generator_decisions(plan, half=0):
    """pix2pix GeneratorPlan (dgan.nets): LeakyReLU of down1-8, ReLU of up1-7, one half."""
    s = plan.s
    rows = slice(half * plan.N, (half + 1) * plan.N)
    out = {}
    for l, (name, _, _, _) in enumerate(plan.downs):
        out[name] = _pos(plan.z_view(s, l)[rows])
    for u, (name, _, co, _) in enumerate(plan.ups):
        out[name] = _pos(s["cat"][u][..., :co][rows])
    return out


def discriminator_decisions(plan, half=0):
    """pix2pix DiscriminatorPlan: LeakyReLU of down1-3 and conv, one half (0 real, 1 fake)."""
    rows = slice(half * plan.N, (half + 1) * plan.N)
    return {name: _pos(z[rows]) for (name, _, _, _), z in zip(plan.specs, plan.z)}


def to_oracle(masks):
    """oracle.decisions.Decisions over exported masks."""
    from oracle.decisions import Decisions
    t = lambda v: torch.from_numpy(np.ascontiguousarray(v))
    return Decisions({k: (t(v[0]), t(v[1])) if isinstance(v, tuple) else t(v) for k, v in masks.items()})


def audit_ok(decs, tie_tol, what=""):
    """Every overridden decision is a near-tie: |fp64 pre-activation| (or the gap
    to the window maximum) below tie_tol of the layer's scale.  Returns the
    total number of overridden elements."""
    tot = 0
    for label, d in decs.items():
        n, worst, where = d.worst()
        tot += n
        assert worst <= tie_tol, (f"{what} {label}: decision at {where} differs from the oracle's on a value "
                                  f"{worst:.2e} of the layer scale from the tie (> {tie_tol:.0e})")
    return tot
