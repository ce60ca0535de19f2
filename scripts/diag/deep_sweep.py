#!/usr/bin/env python3
"""Split-K / tile sweep of the deep U-Net layers' conv ops (pix2pix bs16, batched
2N = 32 passes; down6-8, up1-3), bf16x6 and fp32 MFMA paths: HIP-event time per
call for every (math, tile config, split count) the planner can take, beside the
planner's own choice.  DG_FORCE_X6CFG / DG_FORCE_CFG / DG_FORCE_SPLITS at plan time.

    python scripts/diag/deep_sweep.py > profiles/r3/deep_sweep.txt
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]

import torch  # noqa: E402

LAYERS = [
    # name, N, H, W, Cin, Cout, transpose
    ("G.down6", 32, 8, 8, 512, 512, False),
    ("G.down7", 32, 4, 4, 512, 512, False),
    ("G.down8", 32, 2, 2, 512, 512, False),
    ("G.up1", 32, 1, 1, 512, 512, True),
    ("G.up2", 32, 2, 2, 1024, 512, True),
    ("G.up3", 32, 4, 4, 1024, 512, True),
]
OPS = ("fwd", "bwd_data", "bwd_filter")
X6_CFGS = range(6)
F32_CFGS = range(7)
SPLITS = (1, 2, 4, 8, 16, 32, 64, 128)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


def one(L, op, math, cfg, splits, ws):
    from dgan import ops
    name, N, H, W, Ci, Co, tr = L
    for k in ("DG_FORCE_X6CFG", "DG_FORCE_CFG", "DG_FORCE_SPLITS"):
        os.environ.pop(k, None)
    if cfg is not None:
        os.environ["DG_FORCE_X6CFG" if math == "bf16x6" else "DG_FORCE_CFG"] = str(cfg)
    if splits is not None:
        os.environ["DG_FORCE_SPLITS"] = str(splits)
    try:
        d = ops.ConvDesc(N, H, W, Ci, Co, 4, 2, "same", tr, math=math)
    finally:
        for k in ("DG_FORCE_X6CFG", "DG_FORCE_CFG", "DG_FORCE_SPLITS"):
            os.environ.pop(k, None)
    x = torch.randn(N, H, W, Ci, device="cuda")
    w = torch.randn(*d.weight_shape, device="cuda") * 0.05
    dy = torch.randn(N, d.Ho, d.Wo, Co, device="cuda")
    y = torch.empty(N, d.Ho, d.Wo, Co, device="cuda")
    dx = torch.empty_like(x)
    dw = torch.empty_like(w)
    fn = {"fwd": lambda: d.fwd(x, w, y, ws=ws), "bwd_data": lambda: d.bwd_data(dy, w, dx, ws=ws),
          "bwd_filter": lambda: d.bwd_filter(x, dy, dw, ws=ws)}[op]
    return timeit(fn)


def main():
    from dgan.ops import Workspace
    ws = Workspace(torch.device("cuda"))
    for L in LAYERS:
        for op in OPS:
            base = one(L, op, None, None, None, ws)
            best = (base, "planner")
            for math, cfgs in (("bf16x6", X6_CFGS), ("fp32", F32_CFGS)):
                for cfg in cfgs:
                    for sp in SPLITS:
                        try:
                            t = one(L, op, math, cfg, sp, ws)
                        except Exception:
                            continue
                        if t < best[0]:
                            best = (t, f"{math} cfg {cfg} splits {sp}")
            print(f"{L[0]:8s} {op:10s} planner {base:7.1f} us   best {best[0]:7.1f} us  ({best[1]})", flush=True)


if __name__ == "__main__":
    main()
