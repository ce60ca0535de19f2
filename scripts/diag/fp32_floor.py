#!/usr/bin/env python3
"""fp32 noise floor of the headline step (test infrastructure, CPU only): the torch
restatement (oracle/torch_p2p.py) in fp32 vs fp64, the fp32 run taking the fp64 run's
ReLU / LeakyReLU / max-pool decisions, so only arithmetic differs.  pix2pix full width,
bs2 256x256, dropout 0.5, identity pass, VGG19 content loss (seeded stand-in weights).
Output: profiles/r3/fp32_floor_full_width.txt."""
import os
import sys

import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO, os.path.join(REPO, "scripts")]
torch.set_num_threads(os.cpu_count())
from oracle import p2p_oracle as O
from oracle import torch_p2p as T
from oracle.decisions import Decisions
from dgan.nets import d_variables, g_variables, init_variables
from gen_golden import vgg_weights

class Rec(Decisions):
    def __init__(self):
        super().__init__(); self.rec = {}
    def relu(self, name, x):
        self.rec[name] = (x.detach() > 0).numpy().copy(); return super().relu(name, x)
    def lrelu(self, name, x, a):
        self.rec[name] = (x.detach() > 0).numpy().copy(); return super().lrelu(name, x, a)
    def prelu(self, name, x, a):
        self.rec[name] = (x.detach() > 0).numpy().copy(); return super().prelu(name, x, a)
    def maxpool2(self, name, x):
        N, H, W, C = x.shape
        win = x.detach()[:, :H//2*2, :W//2*2].reshape(N, H//2, 2, W//2, 2, C).permute(0,1,3,5,2,4).reshape(N, H//2, W//2, C, 4)
        self.rec[name] = win.argmax(-1).numpy().copy(); return super().maxpool2(name, x)

seed = 5
G = init_variables(g_variables(1), seed); D = init_variables(d_variables(1), seed + 1)
PV = vgg_weights(seed + 7)
x, y = O.synthetic_pair(2, 256, seed=21)
keys = ["Gx", "Gy", "Dr", "Df", "Vsr", "Vhr"]
recs = {k: Rec() for k in keys}
r64 = T.step_grads(G, D, x, y, width=1, drop_rate=0.5, drop_seed=4, PV=PV, dtype=torch.float64, dec=recs)
dec = {k: Decisions(recs[k].rec) for k in keys}
r32 = T.step_grads(G, D, x, y, width=1, drop_rate=0.5, drop_seed=4, PV=PV, dtype=torch.float32, dec=dec)
print("overrides", {k: sum(v[0] for v in dec[k].audit.values()) for k in keys})
for lab, a, b in (("G", r64[1], r32[1]), ("D", r64[2], r32[2])):
    rows = []
    for k in a:
        e = np.abs(a[k] - b[k]).max(); m = np.abs(a[k]).max()
        rows.append((e, k, m))
    rows.sort(reverse=True)
    for e, k, m in rows:
        print(f"{lab} {k:28s} err {e:.3e} max {m:.3e} rel {e/m:.2e}")
    print(f"{lab}: {sum(e > 1e-4 for e, _, _ in rows)} of {len(rows)} variables above 1e-4; "
          f"max err / max|g| {max(e / m for e, _, m in rows if m > 0):.2e}")
