"""One-off: loss-scale state and gradient finiteness of an SRGAN fp16 step."""
import os, sys
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO, os.path.join(REPO, "tests")]
from test_fp16_gpu import Args, _synthetic
from srgan import SRGAN
for big in (False, True):
    m = SRGAN(Args(crop_size=32, vgg_width=8))
    x, y = _synthetic(2, 32, 4, seed=3)
    tr = m.trainer(x.shape, y.shape)
    lsg, lsd = m.loss_scales
    if big:
        lsg[0] = 3.0e38
    xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    tr.G.plan  # noqa
    tr.step(xd, yd, apply=False)
    torch.cuda.synchronize()
    print("big", big, "lsg", lsg.tolist(), "lsd", lsd.tolist())
    for n, _ in m.discriminator.arena.var_list:
        g = m.discriminator.arena.grad_of(n).cpu().numpy()
        print("  D", n, "finite", np.isfinite(g).mean(), "max", np.nanmax(np.abs(g)))
