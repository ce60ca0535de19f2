#!/usr/bin/env python3
"""SRGAN bs32 24->96 in mixed_float16 at Keras' 2^15: one step (apply=False), the finite
flags of both loss scales and the largest |grad| per network (A/B of plan switches via
DG_PLAN_DISABLE)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]

import torch  # noqa: E402


def main():
    from bench import Args, WORKLOADS, synthetic_batch
    from srgan import SRGAN
    wl = WORKLOADS["srgan"]
    m = SRGAN(Args(crop_size=96, scale=4, lr=1e-3, fp16=1, retrain=0, seed=21))
    x, y = (torch.from_numpy(t).cuda() for t in synthetic_batch(wl, 32, 61))
    tr = m.trainer(x.shape, y.shape)
    tr.step(x, y, apply=False)
    torch.cuda.synchronize()
    lg, ld = m.loss_scales
    gG, gD = m.generator.arena.grad, m.discriminator.arena.grad
    bad = {}
    for net in (m.generator, m.discriminator):
        for n, _ in net.arena.var_list:
            g = net.arena.grad_of(n)
            if not torch.isfinite(g).all():
                bad[n] = int((~torch.isfinite(g)).sum())
    print(os.environ.get("DG_PLAN_DISABLE", "-"), "flags", float(lg[2]), float(ld[2]), "max|gG|",
          float(gG[torch.isfinite(gG)].abs().max()), "max|gD|", float(gD[torch.isfinite(gD)].abs().max()),
          "non-finite:", dict(list(bad.items())[:8]), flush=True)


if __name__ == "__main__":
    main()
