"""Activation decisions of a forward pass -- TEST INFRASTRUCTURE ONLY.

A ReLU / LeakyReLU / PReLU picks a slope per element (x > 0 or not) and a
2x2 max pool picks one element per window.  These are discrete functions of
the pre-activation values, so where fp32 (the HIP path) and fp64 (the oracle)
put a value on different sides of a tie -- |x| within fp32 rounding of 0, or
two window entries within rounding of each other -- the two backwards route
the gradient differently and no elementwise tolerance can compare them.

`Decisions` lets the fp64 oracle take the GPU's decisions instead of its own
("mask-conditioned" parity): every activation site, keyed by its Keras layer
name, uses the mask (or max-pool argmax) exported from the HIP path's
activation buffers.  Each override is audited: an element may only differ
from the oracle's own decision when it is a near-tie, i.e. its fp64
pre-activation is within `tie_tol` of zero (of the window maximum for a
pool) relative to that layer's scale.  Tests assert the audit, so a GPU
indexing bug cannot hide behind a forced mask: a wrong decision on a value
that is not a near-tie fails the audit.

With no forced decisions the functions are the plain TF semantics
(relu grad 0 at 0, LeakyReLU grad alpha at 0, max pool to the first
maximum), i.e. identical to oracle/sr_oracle.py and oracle/torch_p2p.py.
"""
import torch
import torch.nn.functional as F


class Decisions:
    """forced: {layer name: bool mask (activation sites, the activation's
    output shape) or int argmax in 0..3 (max-pool sites, row-major 2x2 window
    index, the pool's output shape)}, numpy or torch, or a (decisions, known)
    pair of which only the `known` elements are forced (a conv whose max pool
    ran in its epilogue exports its ReLU decision at the pooled element only).
    Sites without an entry use the oracle's own decision."""

    def __init__(self, forced=None):
        self.forced = dict(forced or {})
        self.audit = {}   # name -> (n_overridden, worst |tie| / layer scale)

    def _take(self, name, own, tie, scale):
        f = self.forced.get(name)
        if f is None:
            return own
        known = None
        if isinstance(f, tuple):   # (decisions, where they are known): the oracle's own elsewhere
            f, known = f
            known = torch.as_tensor(known).to(own.device).reshape(own.shape)
        f = torch.as_tensor(f).to(own.device).reshape(own.shape)
        if f.dtype != own.dtype:
            f = f.to(own.dtype)
        if known is not None:
            f = torch.where(known, f, own)
        diff = f != own
        n = int(diff.sum())
        worst = float(tie[diff].max() / scale) if n else 0.0
        self.audit[name] = (n, worst)
        return f

    def _mask(self, name, x):
        xd = x.detach()
        own = xd > 0
        scale = max(float(xd.abs().max()), 1e-300)
        return self._take(name, own, xd.abs(), scale)

    def relu(self, name, x):
        if name not in self.forced:
            return F.relu(x)
        return x * self._mask(name, x).to(x.dtype)

    def lrelu(self, name, x, alpha):
        if name not in self.forced:
            return torch.where(x > 0, x, alpha * x)
        return torch.where(self._mask(name, x), x, alpha * x)

    def prelu(self, name, x, alpha):
        """PReLU(shared_axes=[1, 2]): relu(x) - alpha * relu(-x)."""
        a = alpha.reshape(-1)
        if name not in self.forced:
            return F.relu(x) - a * F.relu(-x)
        return torch.where(self._mask(name, x), x, a * x)

    def maxpool2(self, name, x):
        """MaxPool2D(2, 2) on NHWC; the gradient goes to ONE element per
        window (TF MaxPoolGrad: the forward argmax, first maximum in
        row-major window order)."""
        N, H, W, C = x.shape
        x = x[:, :H // 2 * 2, :W // 2 * 2]
        win = x.reshape(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 5, 2, 4).reshape(N, H // 2, W // 2, C, 4)
        wd = win.detach()
        own = wd.argmax(dim=-1)
        if name in self.forced:
            mx = wd.max(dim=-1).values
            tie = (mx.unsqueeze(-1) - wd).gather(-1, torch.as_tensor(self.forced[name]).reshape(own.shape)
                                                 .to(torch.int64).unsqueeze(-1))[..., 0]
            scale = max(float(wd.abs().max()), 1e-300)
            idx = self._take(name, own, tie, scale)
        else:
            idx = own
        return win.gather(-1, idx.to(torch.int64).unsqueeze(-1))[..., 0]

    def worst(self):
        """(total overridden elements, worst tie ratio, layer of the worst)."""
        tot, w, where = 0, 0.0, None
        for k, (n, r) in self.audit.items():
            tot += n
            if r > w:
                w, where = r, k
        return tot, w, where


PLAIN = Decisions()


def of(dec):
    return PLAIN if dec is None else dec
