#!/usr/bin/env python3
"""Time single conv ops of the pix2pix bs16 step under each bf16x6 tile config
(DG_FORCE_X6CFG at plan time) against the planner's own choice.

    python scripts/diag/cfg_sweep.py [--iters 10] [--cfgs 0,1,4,5,6]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]

import torch  # noqa: E402

LAYERS = [
    # name, N, H, W, Cin, Cout, k, s, transpose, ops
    ("G.up7", 32, 64, 64, 256, 64, 4, 2, True, ("fwd", "bwd_data", "bwd_filter")),
    ("G.down2", 32, 128, 128, 64, 128, 4, 2, False, ("fwd", "bwd_data", "bwd_filter")),
    ("D.down2.half", 16, 128, 128, 64, 128, 4, 2, False, ("bwd_data",)),
    ("G.up6", 32, 32, 32, 512, 128, 4, 2, True, ("fwd",)),
    ("V.b2c1", 16, 128, 128, 64, 128, 3, 1, False, ("bwd_data",)),
]


def timeit(fn, iters):
    for _ in range(2):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def run_layer(L, op, cfg, iters):
    from dgan import ops
    name, N, H, W, Ci, Co, k, s, tr, _ = L
    if cfg is None:
        os.environ.pop("DG_FORCE_X6CFG", None)
    else:
        os.environ["DG_FORCE_X6CFG"] = str(cfg)
    d = ops.ConvDesc(N, H, W, Ci, Co, k, s, "same", tr)
    x = torch.randn(N, H, W, Ci, device="cuda")
    w = torch.randn(*d.weight_shape, device="cuda") * 0.05
    dy = torch.randn(N, d.Ho, d.Wo, Co, device="cuda")
    if op == "fwd":
        y = torch.empty(d.out_shape, device="cuda")
        f = lambda: d.fwd(x, w, y)
    elif op == "bwd_data":
        dx = torch.empty_like(x)
        f = lambda: d.bwd_data(dy, w, dx)
    else:
        dw = torch.empty_like(w)
        f = lambda: d.bwd_filter(x, dy, dw)
    t = timeit(f, iters)
    os.environ.pop("DG_FORCE_X6CFG", None)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--cfgs", default="0,1,4,5,6")
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    for L in LAYERS:
        for op in L[-1]:
            row = [f"{L[0]:13s} {op:10s} plan {run_layer(L, op, None, a.iters):7.1f}"]
            for c in cfgs:
                row.append(f"c{c} {run_layer(L, op, c, a.iters):7.1f}")
            print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
