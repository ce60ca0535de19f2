#!/usr/bin/env python3
"""Two fresh pix2pix bs16 models, one step each (apply=False): are the generator output, the
losses and the gradients bit-identical?  Reports the first tensors that differ and by how much
(the run-to-run determinism tests/test_fullsize_gpu.py asserts).  Environment switches of the
library / trainer apply as usual, so a same-box comparison of configurations is
    for e in "" DG_NO_OVERLAP=1 DG_XCD_NG=0; do env $e python scripts/diag/determinism.py; done
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]

import torch  # noqa: E402


class Args:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def run(content, reps):
    from dataloader import synthetic_pair
    from pix2pix import Pix2Pix
    x, y = synthetic_pair(16, 256, 4)
    x, y = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
    outs = []
    for _ in range(reps):
        m = Pix2Pix(Args(crop_size=256, width=1, seed=3, dropout_seed=1, retrain=0, content_loss=int(content)))
        tr = m.trainer(x.shape)
        loss = tr.step(x, y, apply=False).clone()
        torch.cuda.synchronize()
        outs.append({"loss": loss, "gen": tr.gout.clone(), "logits": tr.D.logits.clone(),
                     "gG": m.generator.arena.grad.clone(), "gD": m.discriminator.arena.grad.clone()})
        del m, tr
        torch.cuda.empty_cache()
    base = outs[0]
    for i, o in enumerate(outs[1:], 1):
        diff = {k: float((o[k] - base[k]).abs().max()) for k in base if not torch.equal(o[k], base[k])}
        print(f"content={int(content)} rep {i}: " + ("identical" if not diff else f"DIFFER {diff}"), flush=True)


if __name__ == "__main__":
    for c in [int(v) for v in os.environ.get("CONTENT", "0,1").split(",")]:
        run(c, int(os.environ.get("REPS", "3")))
