#!/usr/bin/env python3
"""The deep U-Net layers' conv ops (pix2pix bs16, 2N = 32) on the planner's own
plans, 20 calls each, for a rocprofv3 --kernel-trace of their kernels."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from deep_sweep import LAYERS, OPS  # noqa: E402


def main():
    from dgan import ops
    ws = ops.Workspace(torch.device("cuda"))
    for name, N, H, W, Ci, Co, tr in LAYERS:
        d = ops.ConvDesc(N, H, W, Ci, Co, 4, 2, "same", tr)
        x = torch.randn(N, H, W, Ci, device="cuda")
        w = torch.randn(*d.weight_shape, device="cuda") * 0.05
        dy = torch.randn(N, d.Ho, d.Wo, Co, device="cuda")
        y = torch.empty(N, d.Ho, d.Wo, Co, device="cuda")
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        for op in OPS:
            fn = {"fwd": lambda: d.fwd(x, w, y, ws=ws), "bwd_data": lambda: d.bwd_data(dy, w, dx, ws=ws),
                  "bwd_filter": lambda: d.bwd_filter(x, dy, dw, ws=ws)}[op]
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            print(name, op, flush=True)


if __name__ == "__main__":
    main()
