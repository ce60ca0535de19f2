#!/usr/bin/env python3
"""Per-layer timing of the conv engine on the pix2pix bs16 shapes (HIP events,
median of reps), with the per-step call multiplicity of the fused train step,
so kernel changes can be A/B'd quickly.  Prints one line per (layer, op)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "denoise-gan_amd"))

import torch  # noqa: E402
from dgan.ops import ConvDesc, Workspace  # noqa: E402

B = int(os.environ.get("DG_BS", "16"))
MATH = os.environ.get("DG_MATH")   # conv arithmetic ("f16x3", "bf16x6", ...); unset: the planner's default
# (name, H, W, Cin, Cout, k, s, pad, transpose, calls fwd, bwd_data, bwd_filter per train step)
LAYERS = [
    ("G.down1", 256, 256, 3, 64, 4, 2, "same", False, (2, 0, 2)),
    ("G.down2", 128, 128, 64, 128, 4, 2, "same", False, (2, 2, 2)),
    ("G.down3", 64, 64, 128, 256, 4, 2, "same", False, (2, 2, 2)),
    ("G.down4", 32, 32, 256, 512, 4, 2, "same", False, (2, 2, 2)),
    ("G.down5", 16, 16, 512, 512, 4, 2, "same", False, (2, 2, 2)),
    ("G.down6", 8, 8, 512, 512, 4, 2, "same", False, (2, 2, 2)),
    ("G.down7", 4, 4, 512, 512, 4, 2, "same", False, (2, 2, 2)),
    ("G.down8", 2, 2, 512, 512, 4, 2, "same", False, (2, 2, 2)),
    ("G.up1", 1, 1, 512, 512, 4, 2, "same", True, (2, 2, 2)),
    ("G.up2", 2, 2, 1024, 512, 4, 2, "same", True, (2, 2, 2)),
    ("G.up3", 4, 4, 1024, 512, 4, 2, "same", True, (2, 2, 2)),
    ("G.up4", 8, 8, 1024, 512, 4, 2, "same", True, (2, 2, 2)),
    ("G.up5", 16, 16, 1024, 256, 4, 2, "same", True, (2, 2, 2)),
    ("G.up6", 32, 32, 512, 128, 4, 2, "same", True, (2, 2, 2)),
    ("G.up7", 64, 64, 256, 64, 4, 2, "same", True, (2, 2, 2)),
    ("G.last", 128, 128, 128, 3, 4, 2, "same", True, (2, 2, 2)),
    ("D.down1", 256, 256, 6, 64, 4, 2, "same", False, (2, 1, 2)),
    ("D.down2", 128, 128, 64, 128, 4, 2, "same", False, (2, 3, 2)),
    ("D.down3", 64, 64, 128, 256, 4, 2, "same", False, (2, 3, 2)),
    ("D.conv", 32, 32, 256, 512, 4, 1, (1, 1, 1, 1), False, (2, 3, 2)),
    ("D.last", 31, 31, 512, 1, 4, 1, (1, 1, 1, 1), False, (2, 3, 2)),
    # VGG19 to block5_conv4 on 256x256 (content loss: fwd on G(x) and y, bwd_data on G(x))
    ("V.b1c1", 256, 256, 3, 64, 3, 1, "same", False, (2, 1, 0)),
    ("V.b1c2", 256, 256, 64, 64, 3, 1, "same", False, (2, 1, 0)),
    ("V.b2c1", 128, 128, 64, 128, 3, 1, "same", False, (2, 1, 0)),
    ("V.b2c2", 128, 128, 128, 128, 3, 1, "same", False, (2, 1, 0)),
    ("V.b3c1", 64, 64, 128, 256, 3, 1, "same", False, (2, 1, 0)),
    ("V.b3cx", 64, 64, 256, 256, 3, 1, "same", False, (6, 3, 0)),
    ("V.b4c1", 32, 32, 256, 512, 3, 1, "same", False, (2, 1, 0)),
    ("V.b4cx", 32, 32, 512, 512, 3, 1, "same", False, (6, 3, 0)),
    ("V.b5cx", 16, 16, 512, 512, 3, 1, "same", False, (8, 4, 0)),
]


def main():
    only = os.environ.get("DG_LAYERS")
    reps = int(os.environ.get("DG_REPS", "10"))
    dev = torch.device("cuda")
    ws = Workspace(dev)
    tot_ms, tot_fl = 0.0, 0.0
    rows = []
    for name, H, W, ci, co, k, s, pad, tr, calls in LAYERS:
        if only and name not in only.split(","):
            continue
        d = ConvDesc(B, H, W, ci, co, k, s, pad, tr, **({"math": MATH} if MATH else {}))
        x = torch.randn(B, H, W, ci, device=dev)
        w = torch.randn(*d.weight_shape, device=dev) * 0.02
        y = torch.empty(d.out_shape, device=dev)
        dy = torch.randn(d.out_shape, device=dev)
        dx = torch.empty_like(x)
        dw = torch.empty_like(w)
        ops = [("fwd", lambda: d.fwd(x, w, y, ws=ws)), ("bwd_data", lambda: d.bwd_data(dy, w, dx, ws=ws)),
               ("bwd_filter", lambda: d.bwd_filter(x, dy, dw, ws=ws))]
        for (op, fn), n in zip(ops, calls):
            if n == 0:
                continue
            for _ in range(3):
                fn()
            times = []
            for _ in range(reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                times.append(e0.elapsed_time(e1))
            ms = sorted(times)[len(times) // 2]
            tf = d.flops / (ms * 1e-3) / 1e12
            tot_ms += ms * n
            tot_fl += d.flops * n
            rows.append(dict(layer=name, op=op, ms=round(ms, 4), tflops=round(tf, 1), calls=n))
            print(f"{name:8s} {op:10s} {ms:8.4f} ms {tf:7.1f} TF/s  x{n}", flush=True)
    print(json.dumps({"conv_ms_per_step": round(tot_ms, 3), "tflops": round(tot_fl / (tot_ms * 1e-3) / 1e12, 2)}))


if __name__ == "__main__":
    main()
