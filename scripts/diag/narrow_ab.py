#!/usr/bin/env python3
"""Same-box A/B of the two narrow-output (Co 1 / 3) forward kernels over the
SR family's narrow layers at their BASELINE batch sizes: the thread-per-pixel
k_narrow_fwd_px (default) vs the wave-per-pixel k_narrow_fwd
(DG_PLAN_DISABLE=narrow_px).  HIP events, median of reps, alternating A/B
rounds.  Sets csrc/conv.hip NFWD_PX_MIN_M."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "denoise-gan_amd"))

import torch  # noqa: E402
from dgan.ops import ConvDesc, Workspace  # noqa: E402

LAYERS = [
    # (name, N, H, W, Cin, Cout, k)
    ("fsrgan.conv2d_out bs8", 8, 512, 512, 32, 3, 3),
    ("srgan.conv2d_out bs32", 32, 96, 96, 64, 3, 1),
    ("ae.conv11 bs4", 4, 64, 64, 32, 3, 3),
    ("fsrgan.D.logits bs8", 8, 32, 32, 64, 1, 1),
    ("srgan.D.logits bs32", 32, 6, 6, 64, 1, 1),
    ("ae.D.logits bs4", 4, 4, 4, 64, 1, 1),
]


def time_fwd(d, x, w, b, y, ws, reps):
    for _ in range(3):
        d.fwd(x, w, y, bias=b, ws=ws)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        d.fwd(x, w, y, bias=b, ws=ws)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def main():
    reps = int(os.environ.get("DG_REPS", "30"))
    dev = torch.device("cuda")
    ws = Workspace(dev)
    for name, N, H, W, ci, co, k in LAYERS:
        d = ConvDesc(N, H, W, ci, co, k, 1, "same")
        x = torch.randn(N, H, W, ci, device=dev)
        w = torch.randn(*d.weight_shape, device=dev) * 0.05
        b = torch.randn(co, device=dev)
        y = torch.empty(d.out_shape, device=dev)
        res = {"px": [], "wave": []}
        for _ in range(2):
            for tag in ("px", "wave"):
                if tag == "wave":
                    os.environ["DG_PLAN_DISABLE"] = "narrow_px"
                else:
                    os.environ.pop("DG_PLAN_DISABLE", None)
                res[tag].append(time_fwd(d, x, w, b, y, ws, reps))
        os.environ.pop("DG_PLAN_DISABLE", None)
        M = N * d.out_shape[1] * d.out_shape[2]
        px, wv = min(res["px"]), min(res["wave"])
        print(f"{name:24s} M {M:9d}  px {px * 1e3:9.1f} us  wave {wv * 1e3:9.1f} us  wave/px {wv / px:5.2f}",
              flush=True)


if __name__ == "__main__":
    main()
