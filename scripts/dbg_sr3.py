"""Debug: split the trainer's d(gen) into its content and non-content parts vs the oracle."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "denoise-gan_amd"), os.path.join(os.path.dirname(__file__), "..")]
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np, torch
from test_sr_gpu import Args, _synthetic
from oracle import sr_oracle as S

kind = sys.argv[1]
if kind == "fsrgan":
    from fsrgan import FastSRGAN as C; N, H, scale = 2, 64, 4
else:
    from autoencoder import Autoencoder as C; N, H, scale = 4, 64, 1
m = C(Args(crop_size=H, scale=scale))
st = S.SRState(kind, m.generator.arena.export(), m.discriminator.arena.export(), m.vgg.arena.export(), scale=scale)
PV = {k: torch.tensor(v) for k, v in st.PV.items()}
PD = {k: torch.tensor(v) for k, v in st.PD.items()}
x, y = _synthetic(N, H, H, scale, seed=50)
ref = S.train_step(st, x, y, apply=False)
tr = m.trainer(x.shape, y.shape)
tr.step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), apply=False)
torch.cuda.synchronize()
gen_g = tr.gen_output.cpu().double().numpy()
gen_o = ref["gen"]
print("gen diff", np.abs(gen_g - gen_o).max())
tot = tr.dgen.cpu().double().numpy()
cont_g = 127.5 * tr.content.dpre.cpu().double().numpy()[..., ::-1]
rest_g = tot - cont_g
yt = torch.tensor(y.astype(np.float64))
def parts(gen):
    gt = torch.tensor(gen, requires_grad=True)
    c = S.content_loss(PV, yt, gt)
    dc = torch.autograd.grad(c, gt)[0].numpy()
    gt2 = torch.tensor(gen, requires_grad=True)
    zf = S.sr_discriminator(PD, gt2, S.BNStats())
    # D(fake) is in a batch of its own in BN: same as the step
    rest = 1e-3 * S.bce_logits(zf, 1.0) + (yt - gt2).abs().mean()
    dr = torch.autograd.grad(rest, gt2)[0].numpy()
    return dc, dr
dc_o, dr_o = parts(gen_o)
dc_g, dr_g = parts(gen_g)
print("total vs oracle total", np.abs(tot - ref["dgen"]).max(), "scale", np.abs(ref["dgen"]).max())
print("content part: gpu vs oracle(gen_o)", np.abs(cont_g - dc_o).max(), " vs oracle(gen_gpu)", np.abs(cont_g - dc_g).max())
print("rest part: gpu vs oracle(gen_o)", np.abs(rest_g - dr_o).max(), " vs oracle(gen_gpu)", np.abs(rest_g - dr_g).max())
print("oracle content at gen_o vs gen_gpu", np.abs(dc_o - dc_g).max(), "rest", np.abs(dr_o - dr_g).max())
print("oracle total vs parts", np.abs(ref["dgen"] - dc_o - dr_o).max())
