#!/usr/bin/env python3
"""Tile / split sweep of FastSRGAN's narrow-channel conv ops (bs8 shard, 32-64
channels at 128-512 px): HIP-event time per call for the planner's choice and
every bf16x6 / fp32 tile config at a few split counts (DG_FORCE_X6CFG /
DG_FORCE_CFG / DG_FORCE_SPLITS at plan time), to check the planner's cost model
on these memory-bound shapes.

    python scripts/diag/narrow_sweep.py > profiles/r3/narrow_sweep_fsrgan.txt
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO, os.path.dirname(os.path.abspath(__file__))]

import torch  # noqa: E402
from deep_sweep import timeit  # noqa: E402

LAYERS = [
    # name, N, H, W, Cin, Cout, k, s
    ("D.d2", 8, 512, 512, 32, 32, 3, 2),
    ("D.d3", 8, 256, 256, 32, 32, 3, 1),
    ("D.d4", 8, 256, 256, 32, 32, 3, 2),
    ("D.d5", 8, 128, 128, 32, 64, 3, 1),
    ("G.deconv1", 8, 256, 256, 32, 128, 3, 1),
    ("G.out", 8, 512, 512, 32, 3, 3, 1),
]
OPS = ("fwd", "bwd_data", "bwd_filter")


def one(L, op, math, cfg, splits):
    from dgan import ops
    name, N, H, W, Ci, Co, k, s = L
    keys = ("DG_FORCE_X6CFG", "DG_FORCE_CFG", "DG_FORCE_SPLITS")
    for key in keys:
        os.environ.pop(key, None)
    if cfg is not None:
        os.environ["DG_FORCE_X6CFG" if math == "bf16x6" else "DG_FORCE_CFG"] = str(cfg)
    if splits is not None:
        os.environ["DG_FORCE_SPLITS"] = str(splits)
    try:
        d = ops.ConvDesc(N, H, W, Ci, Co, k, s, "same", math=math)
    finally:
        for key in keys:
            os.environ.pop(key, None)
    ws = ops.Workspace(torch.device("cuda"))
    T = TENSORS[name]
    fn = {"fwd": lambda: d.fwd(T["x"], T["w"], T["y"], ws=ws),
          "bwd_data": lambda: d.bwd_data(T["dy"], T["w"], T["dx"], ws=ws),
          "bwd_filter": lambda: d.bwd_filter(T["x"], T["dy"], T["dw"], ws=ws)}[op]
    return timeit(fn, iters=10)


TENSORS = {}


def main():
    from dgan import ops
    for L in LAYERS:
        name, N, H, W, Ci, Co, k, s = L
        d = ops.ConvDesc(N, H, W, Ci, Co, k, s, "same")
        TENSORS.clear()
        TENSORS[name] = dict(x=torch.randn(N, H, W, Ci, device="cuda"),
                             w=torch.randn(*d.weight_shape, device="cuda") * 0.05,
                             dy=torch.randn(N, d.Ho, d.Wo, Co, device="cuda"),
                             y=torch.empty(N, d.Ho, d.Wo, Co, device="cuda"),
                             dx=torch.empty(N, H, W, Ci, device="cuda"),
                             dw=torch.empty(*d.weight_shape, device="cuda"))
        for op in OPS:
            base = one(L, op, None, None, None)
            res = []
            for math, cfgs in (("bf16x6", range(7)), ("fp32", range(9))):
                for cfg in cfgs:
                    for sp in ((1, 2, 4) if op != "bwd_filter" else (16, 64, 256, 1024)):
                        try:
                            t = one(L, op, math, cfg, sp)
                        except Exception:
                            continue
                        res.append((t, f"{math} cfg {cfg} splits {sp}"))
            res.sort()
            top = "; ".join(f"{t:.1f} us {w}" for t, w in res[:3])
            print(f"{name:10s} {op:10s} planner {base:7.1f} us | best: {top}", flush=True)


if __name__ == "__main__":
    main()
