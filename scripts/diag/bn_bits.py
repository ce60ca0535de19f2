#!/usr/bin/env python3
"""Bit-identity check of the BN kernels across two library builds (same-box A/B of a
refactor that must not change results): `bn_bits.py OUT.pt` runs BN forward +
backward (fp32 dy, fp16x3 dy planes with their bound) on seeded shapes and saves
every output; `bn_bits.py OUT.pt REF.pt` also compares bitwise with REF.pt.
Load the other build with DG_LIB=<path>."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "denoise-gan_amd"))
import torch  # noqa: E402
from dgan import ops  # noqa: E402

SHAPES = [(1, 4096, 64), (2, 8192, 128), (2, 2048, 512), (1, 300, 96), (2, 64, 1024)]


def run():
    dev = torch.device("cuda")
    out = {}
    for S, M, C in SHAPES:
        g = torch.Generator().manual_seed(S * 7919 + M * 31 + C)
        y = (torch.randn(S * M, C, generator=g) * 1.3 + 0.2).to(dev)
        dz = torch.randn(S * M, C, generator=g).to(dev)
        gm = (1 + 0.2 * torch.randn(C, generator=g)).to(dev)
        bt = (0.1 * torch.randn(C, generator=g)).to(dev)
        mm, mv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        mean, inv = torch.empty(S, C, device=dev), torch.empty(S, C, device=dev)
        z = torch.empty_like(y)
        ops.bn_fwd_train(y, gm, bt, mean, inv, mm, mv, z, act="leaky_relu", alpha=0.3, segments=S)
        dy = torch.empty_like(y)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        ops.bn_bwd(dz, z, y, gm, mean, inv, dy, dg, db, act="leaky_relu", alpha=0.3, segments=S)
        key = f"{S}x{M}x{C}"
        out.update({f"{key}.{n}": t.cpu() for n, t in
                    (("z", z), ("mean", mean), ("inv", inv), ("mm", mm), ("mv", mv), ("dy", dy), ("dg", dg),
                     ("db", db))})
        if C % 32 == 0:
            planes = torch.zeros(S * M * C * 4, dtype=torch.uint8, device=dev)
            bound = ops.max_slot(device=dev)
            dg2, db2 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
            ops.bn_bwd(dz, z, y, gm, mean, inv, dy, dg2, db2, act="leaky_relu", alpha=0.3, segments=S,
                       dy_planes=planes, dy_bound=bound)
            out[f"{key}.planes"] = planes.cpu()
            out[f"{key}.bound"] = bound.cpu()
    torch.cuda.synchronize()
    return out


def main():
    out = run()
    torch.save(out, sys.argv[1])
    if len(sys.argv) > 2:
        ref = torch.load(sys.argv[2], weights_only=True)
        bad = [k for k in out if not torch.equal(out[k], ref[k])]
        print(f"{len(out)} tensors compared, {len(bad)} differ: {bad}")
        sys.exit(1 if bad else 0)
    print(f"{len(out)} tensors saved")


if __name__ == "__main__":
    main()
