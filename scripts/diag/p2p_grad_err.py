"""Per-variable gradient error of one pix2pix step vs the fp64 oracle (diagnostic; the
conv math of G / D from DG_P2P_MATH): python scripts/diag/p2p_grad_err.py [width batch]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]
from oracle import p2p_oracle as O  # noqa: E402
from pix2pix import Pix2Pix  # noqa: E402

width = int(sys.argv[1]) if len(sys.argv) > 1 else 1
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 2


class Args:
    crop_size = 256
    retrain = 0
    content_loss = 0
    width = 1
    seed = 42
    dropout_seed = 5
    dropout_rate = 0.5
    identity_loss = 1


Args.width = width
st = O.P2PState(width=width, seed=42, drop_rate=0.5, drop_seed=5, identity=True)
x, y = O.synthetic_pair(batch, 256, seed=9)
ref = O.train_step(st, x, y, return_grads=True, apply=False)
m = Pix2Pix(Args())
tr = m.trainer(x.shape)
tr.step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), apply=False)
torch.cuda.synchronize()
for label, arena, g in (("G", m.generator.arena, ref["gG"]), ("D", m.discriminator.arena, ref["gD"])):
    rows = []
    for name, g_ref in g.items():
        got = arena.grad_of(name).detach().double().cpu().numpy()
        err = float(np.abs(got - g_ref).max())
        rows.append((err, name, err / (np.abs(g_ref).max() + 1e-30),
                     float(np.linalg.norm(got - g_ref) / (np.linalg.norm(g_ref) + 1e-30))))
    rows.sort(reverse=True)
    for e, n, r, l2 in rows[:8]:
        print(f"{label} {n:22s} max-abs {e:.3e} rel-max {r:.3e} rel-L2 {l2:.3e}")
