"""Debug: VGG19 content-loss gradient vs the oracle at several sizes."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "denoise-gan_amd"), os.path.join(os.path.dirname(__file__), "..")]
import numpy as np, torch
from oracle import sr_oracle as S
from dgan.sr_trainer import VGGNetwork, ContentLoss
from dgan import ops
from dataloader import synthetic_pair

vgg = VGGNetwork(seed=11)
PV = {k: torch.tensor(v.astype(np.float64)) for k, v in vgg.arena.export().items()}
for N, H in ((2, 32), (2, 64), (1, 64), (4, 32), (2, 48)):
    x, y = synthetic_pair(N, H, seed=3)
    gen = np.tanh(np.arctanh(np.clip(y, -0.99, 0.99)) + 0.3 * np.random.default_rng(0).standard_normal(y.shape)).astype(np.float32)
    gt = torch.tensor(gen.astype(np.float64), requires_grad=True)
    c = S.content_loss(PV, torch.tensor(y.astype(np.float64)), gt)
    d0 = torch.autograd.grad(c, gt)[0].numpy()
    cl = ContentLoss(vgg, N, H, H, torch.device("cuda"))
    ws = ops.Workspace(); ws.get(cl.ws_bytes)
    dg = torch.zeros((N, H, H, 3), device="cuda")
    v = cl.forward(torch.from_numpy(gen).cuda(), torch.from_numpy(y).cuda(), ws=ws)
    cl.backward(dg, beta=0.0, ws=ws)
    torch.cuda.synchronize()
    d = dg.cpu().double().numpy()
    e = np.abs(d - d0)
    print(f"N={N} H={H} content {v.item():.7f} ref {c.item():.7f}  dgen err {e.max():.3e} scale {np.abs(d0).max():.3e} "
          f"frac>1e-3 {(e > 1e-3 * np.abs(d0).max()).mean():.4f}", flush=True)
    if e.max() > 1e-4 * np.abs(d0).max():
        idx = np.unravel_index(np.argmax(e), e.shape)
        print("   worst at", idx)
