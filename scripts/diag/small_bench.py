#!/usr/bin/env python3
"""Time the small-Cin conv ops (conv_small.hip) at the pix2pix bs16 geometry,
with and without the bf16x6 output planes, against the generic GEMM path
(DG_PLAN_DISABLE=small at plan time).  HIP events around N calls of each op.

    python scripts/diag/small_bench.py [--iters 20]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]

import torch  # noqa: E402

LAYERS = [
    # name, N, H, W, Cin, Cout, transpose
    ("G.down1", 32, 256, 256, 3, 64, False),
    ("D.down1", 32, 256, 256, 6, 64, False),
    ("G.last", 32, 128, 128, 128, 3, True),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def run(iters, generic):
    from dgan import ops
    if generic:
        os.environ["DG_PLAN_DISABLE"] = "small"
    else:
        os.environ.pop("DG_PLAN_DISABLE", None)
    out = {}
    for name, N, H, W, Ci, Co, tr in LAYERS:
        d = ops.ConvDesc(N, H, W, Ci, Co, 4, 2, "same", tr)
        x = torch.randn(N, H, W, Ci, device="cuda")
        w = torch.randn(*d.weight_shape, device="cuda") * 0.05
        dy = torch.randn(N, d.Ho, d.Wo, Co, device="cuda")
        y = torch.empty(d.out_shape, device="cuda")
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        r = {}
        r["fwd"] = timeit(lambda: d.fwd(x, w, y, act="lrelu", alpha=0.3), iters)
        if not tr:
            pb = ops.PlaneBuf(6 * y.numel())
            pl = ops.ConvPlanes(fwd_out=pb)
            r["fwd+planes"] = timeit(lambda: d.fwd(x, w, y, act="lrelu", alpha=0.3, planes=pl), iters)
        r["bwd_data"] = timeit(lambda: d.bwd_data(dy, w, dx), iters)
        r["bwd_filter"] = timeit(lambda: d.bwd_filter(x, dy, dw), iters)
        out[name] = r
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    new = run(a.iters, False)
    old = run(a.iters, True)
    for name in new:
        for op, t in new[name].items():
            print(f"{name:8s} {op:11s} small {t:8.1f} us   generic {old[name][op]:8.1f} us")


if __name__ == "__main__":
    main()
