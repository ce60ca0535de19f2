"""Debug: per-variable gradient error table of one SR-family step vs the oracle."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "denoise-gan_amd"), os.path.join(os.path.dirname(__file__), "..")]
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from test_sr_gpu import Args, _synthetic
from oracle import sr_oracle as S

kind = sys.argv[1]
if kind == "fsrgan":
    from fsrgan import FastSRGAN as C; N, H, scale = 2, 64, 4
elif kind == "autoencoder":
    from autoencoder import Autoencoder as C; N, H, scale = 4, 64, 1
else:
    from srgan import SRGAN as C; N, H, scale = 2, 32, 4
kw = {}
if len(sys.argv) > 2:
    kw["content_loss"] = int(sys.argv[2])
m = C(Args(crop_size=H, scale=scale, **kw))
st = S.SRState(kind, m.generator.arena.export(), m.discriminator.arena.export(),
               m.vgg.arena.export() if m.vgg is not None else None, scale=scale)
x, y = _synthetic(N, H, H, scale, seed=50)
ref = S.train_step(st, x, y, apply=False)
tr = m.trainer(x.shape, y.shape)
loss = tr.step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), apply=False)
torch.cuda.synchronize()
print("loss", loss.cpu().numpy(), np.array(ref["losses"]))
d = tr.dgen.cpu().double().numpy(); r = ref["dgen"]
print("dgen err %.3e scale %.3e" % (np.abs(d - r).max(), np.abs(r).max()))
for net, gr in ((m.generator, ref["gG"]), (m.discriminator, ref["gD"])):
    for k, v in gr.items():
        g = net.arena.grad_of(k).cpu().double().numpy()
        e = np.abs(g - v).max(); sc = np.abs(v).max()
        print(f"{k:45s} err {e:.3e} scale {sc:.3e} rel {e / (sc + 1e-30):.2e}")
