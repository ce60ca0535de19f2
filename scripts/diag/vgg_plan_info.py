#!/usr/bin/env python3
"""Which VGG19 activations of the pix2pix content loss (bs16, 256^2) live as planes only, which
convs take the mask from planes (bwd_data_xmask) or from fp32 z (bwd_data_masked), and the
plan arithmetic of each conv op -- a GPU diagnostic (one step)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]
import numpy as np  # noqa: E402
import torch  # noqa: E402


class A:
    crop_size = 256
    retrain = 0
    width = 1
    seed = 1234
    dropout_seed = 0
    identity_loss = 1
    content_loss = 1


def main():
    from pix2pix import Pix2Pix
    from oracle import p2p_oracle as O
    m = Pix2Pix(A())
    x, y = O.synthetic_pair(16, 256, seed=3)
    tr = m.trainer(x.shape)
    tr.step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
    torch.cuda.synchronize()
    c = tr.content
    for name, p in (("fplan", c.fplan), ("tplan", c.tplan), ("bplan", c.bplan)):
        if p is None:
            continue
        nodes = p.graph.nodes if hasattr(p, "graph") else []
        nm = {n.idx: n.name for n in nodes}
        print(name, "nofp32:", sorted(nm.get(i, i) for i in p.nofp32))
        print(name, "premask:", sorted(p.premask) if hasattr(p, "premask") else None)
        print(name, "fused_pool convs:", sorted(nm.get(i, i) for i in getattr(p, "fused_conv", {})))


if __name__ == "__main__":
    main()
