#!/usr/bin/env python3
"""Per-layer conv table of one pix2pix bs16 training step (HIP events per conv
call, dgan.ops.ConvProfile), grouped by layer geometry and op, as a markdown
table: GFLOP, ms, TF/s (fp32-equivalent), the arithmetic of the op's GEMM
(ops.ConvDesc.op_arith) and the fraction of that arithmetic's dense MFMA peak
(fp16x3: bf16 peak / 3 = 838.9 TF/s, bf16x6: / 6 = 419.4, fp16: / 1, fp32 MFMA
157.3), plus each op's own roofline: the larger of its MFMA time at that peak
and its HBM time for the algorithmic fp32 operand bytes (x, w, y once each) at
8 TB/s -- narrow layers (Cin 3/6, Cout 1/3) and the deep U-Net layers (M = 32..512
rows) are HBM- or weight-bound, and `roof` is their fraction of that bound.

    python scripts/layer_table.py [--content 0|1] [--steps 3] > profiles/...md
"""
import argparse
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]

import torch  # noqa: E402

BASIS = 2516.6e12 / 6
HBM = 8.0e12
PEAK = {"fp32": 157.3e12, "bf16x6": 2516.6e12 / 6, "fp16": 2516.6e12, "f16x3": 2516.6e12 / 3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--content", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--model", default="pix2pix", choices=("pix2pix", "srgan", "fsrgan", "autoencoder"))
    ap.add_argument("--fp16", type=int, default=None, help="SR family: mixed_float16 (default: the driver's)")
    a = ap.parse_args()
    from bench import Args, WORKLOADS, synthetic_batch
    from dgan import ops
    wl = WORKLOADS[a.model]
    batch = a.batch or wl["batch"]
    global BASIS
    if a.model == "pix2pix":
        from pix2pix import Pix2Pix
        m = Pix2Pix(Args(crop_size=256, retrain=0, width=1, seed=1234, dropout_seed=0, identity_loss=1,
                         content_loss=a.content))
    else:
        from autoencoder import Autoencoder
        from fsrgan import FastSRGAN
        from srgan import SRGAN
        fp16 = int(wl.get("fp16", 0) if a.fp16 is None else a.fp16)
        if fp16:
            BASIS = 2516.6e12   # fp16 GEMMs: the dense fp16 MFMA peak
        cls = {"srgan": SRGAN, "fsrgan": FastSRGAN, "autoencoder": Autoencoder}[a.model]
        m = cls(Args(crop_size=wl["size"], scale=wl["scale"], lr=1e-3, fp16=fp16, retrain=0, seed=1234,
                     content_loss=a.content))
    x, y = (torch.from_numpy(t).cuda() for t in synthetic_batch(wl, batch, 1000))
    tr = m.trainer(x.shape) if a.model == "pix2pix" else m.trainer(x.shape, y.shape)
    for _ in range(3):
        tr.step(x, y)
    torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    for _ in range(a.steps):
        with ops.ConvProfile() as prof:
            tr.step(x, y)
        torch.cuda.synchronize()
        for r in prof.summary():
            N, H, W, Ci, Co, k, s = r["shape"]
            net, layer = (r["label"] or "?.?").split(".", 1)
            key = (net, layer + (" (T)" if r["transpose"] else ""), r["op"], N, H, W, Ci, Co, k, s, r["arith"])
            agg[key][0] += 1
            agg[key][1] += r["flops"]
            agg[key][2] += r["ms"]
            agg[key][3] += r["bytes"]
    rows = sorted(agg.items(), key=lambda kv: -kv[1][2])
    tot = defaultdict(lambda: [0.0, 0.0, 0.0])
    print(f"| net | layer | op | N | H x W | Cin -> Cout | k/s | arith | calls/step | GFLOP/step | MB/step | ms/step | "
          f"TF/s | frac | bound | roof |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for (net, kind, op, N, H, W, Ci, Co, k, s, ar), (n, fl, ms, by) in rows:
        fl /= a.steps; ms /= a.steps; by /= a.steps
        peak = BASIS if ar == "fp16" and BASIS != PEAK["bf16x6"] else PEAK[ar]
        tot[net][0] += fl; tot[net][1] += ms; tot[net][2] += fl / peak
        tf = fl / (ms * 1e-3) / 1e12
        t_mfma, t_hbm = fl / peak, by / HBM
        bound = "mfma" if t_mfma >= t_hbm else "hbm"
        roof = max(t_mfma, t_hbm) / (ms * 1e-3)
        print(f"| {net} | {kind} | {op} | {N} | {H}x{W} | {Ci}->{Co} | {k}/{s} | {ar} | {n // a.steps} | "
              f"{fl / 1e9:.1f} | {by / 1e6:.0f} | {ms:.3f} | {tf:.1f} | {tf * 1e12 / peak:.3f} | {bound} | {roof:.3f} |")
    print()
    for net, (fl, ms, tp) in sorted(tot.items()):
        tf = fl / (ms * 1e-3) / 1e12
        print(f"- {net}: {fl / 1e9:.1f} GFLOP in {ms:.3f} ms/step = {tf:.1f} TF/s = {tp / (ms * 1e-3):.3f} of its "
              f"ops' arithmetic peaks ({tf * 1e12 / PEAK['bf16x6']:.3f} of the bf16x6 basis)")
    fl = sum(v[0] for v in tot.values()); ms = sum(v[1] for v in tot.values()); tp = sum(v[2] for v in tot.values())
    print(f"- all convs: {fl / 1e9:.1f} GFLOP in {ms:.3f} ms/step = {fl / (ms * 1e-3) / 1e12:.1f} TF/s = "
          f"{tp / (ms * 1e-3):.3f} of the ops' arithmetic peaks ({fl / (ms * 1e-3) / PEAK['bf16x6']:.3f} of the bf16x6 "
          f"basis)")


if __name__ == "__main__":
    main()
