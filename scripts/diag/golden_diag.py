"""One-off: per-variable error of the HIP pix2pix bs16 step vs tests/golden/p2p_bs16.npz."""
import os, sys
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO, os.path.join(REPO, "tests")]
from golden_util import batch, load, names
from pix2pix import Pix2Pix
class A:
    def __init__(s, **k): s.__dict__.update(k)
meta, d = load(sys.argv[1] if len(sys.argv) > 1 else "p2p_bs16")
m = Pix2Pix(A(crop_size=256, retrain=0, width=1, seed=meta["seed"], dropout_seed=meta["drop_seed"], dropout_rate=0.5,
              identity_loss=1, content_loss=int(meta.get("content", 1))))
x, y = batch(meta, meta["batch_seeds"][0])
tr = m.trainer(x.shape)
tr.step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
torch.cuda.synchronize()
for pre, A_ in (("s1|gG|", m.generator.arena), ("s1|gD|", m.discriminator.arena)):
    for n in names(d, pre):
        g = A_.grad_of(n).cpu().double().numpy().ravel()
        idx = d[f"{pre}{n}|idx"]
        err = np.abs(g[idx] - d[f"{pre}{n}|val"]).max()
        l2 = float(d[f"{pre}{n}|l2"]); mx = float(d[f"{pre}{n}|maxabs"])
        print(f"{pre}{n:16s} err {err:.2e} refmax {mx:.2e} l2rel {abs(np.linalg.norm(g)-l2)/l2:.2e}")
