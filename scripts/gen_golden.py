#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ from the fp64
CPU oracles (oracle/p2p_oracle.py, oracle/sr_oracle.py) -- test
infrastructure, run in the build container, never on the GPU box.

    python scripts/gen_golden.py [p2p_bs16] [srgan_bs32] [ae_bs4] [fsrgan_bs8]

The reference ships no tests, fixtures or golden vectors and TensorFlow is
not installable here, so these digests of the oracle at
the BASELINE.json configs are the stable pin the GPU tests
(tests/test_golden_gpu.py) compare the HIP path against, without re-running
the oracle on the box.  Each case is two training steps at the full config:

  step 1   the loss tuple, G(x) (4096 sampled pixels + its PSNR vs y), the
           discriminator logits (full), every G and D gradient (L2 norm,
           max-abs, 64 sampled entries), the BN moving statistics (full)
  step 2   after step 1's Adam update, on a second batch: the loss tuple and
           every parameter after step 2's Adam (64 sampled entries + L2)

Inputs are re-generated from their seeds (dataloader.synthetic_pair); the
weights come from the product's own seeded initialisers (same PCG64
streams), pinned by a crc32 per network so a changed initialiser fails as
"weights differ", not as a parity error.

Cases (BASELINE.json configs):
  p2p_bs16    pix2pix 256x256 bs16, full width, dropout 0.5, identity pass,
              VGG19 content loss (seeded stand-in weights)           configs[1]
  p2p_bs16_core  the same without the content term (the north star's
              "L1 + adversarial" step), other seeds                  configs[1]
  srgan_bs32  SRGAN 4x, 24 -> 96 crops, 16 residual blocks, bs32, VGG19
              content loss                                           configs[2]
  ae_bs4      conv autoencoder 64x64 grayscale (replicated to 3 channels),
              bs4, VGG19 content loss                                configs[0]
  fsrgan_bs8  FastSRGAN 128 -> 512, bs8 (the per-GPU shard of the 8-GPU
              config), VGG19 content loss at 512x512                 configs[4]
"""
import json
import math
import os
import sys
import time
import zlib

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "denoise-gan_amd"))
sys.path.insert(0, REPO)

from dataloader import synthetic_pair  # noqa: E402
from oracle import p2p_oracle as O  # noqa: E402
from oracle import sr_oracle as S  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")
N_SAMPLE = 64
N_GEN_SAMPLE = 4096

CASES = {
    "p2p_bs16": dict(kind="pix2pix", N=16, H=256, scale=1, seed=1234, drop_seed=3, batch_seeds=(1000, 1001),
                     content=1),
    "p2p_bs16_core": dict(kind="pix2pix", N=16, H=256, scale=1, seed=4321, drop_seed=5, batch_seeds=(2000, 2001),
                          content=0),
    "srgan_bs32": dict(kind="srgan", N=32, H=96, scale=4, seed=21, batch_seeds=(50, 51), lr=1e-3),
    "ae_bs4": dict(kind="autoencoder", N=4, H=64, scale=1, seed=21, batch_seeds=(50, 51), lr=1e-3, gray=True),
    "fsrgan_bs8": dict(kind="fsrgan", N=8, H=512, scale=4, seed=21, batch_seeds=(60, 61), lr=1e-3),
}


def sample_idx(key, size, k):
    rng = np.random.default_rng(zlib.crc32(key.encode()))
    return np.sort(rng.choice(size, min(k, size), replace=False)).astype(np.int64)


def weights_crc(params, order):
    c = 0
    for n in order:
        c = zlib.crc32(np.ascontiguousarray(params[n], np.float32).tobytes(), c)
    return c


def psnr(img, ref):
    a = (np.asarray(img, np.float64) + 1) / 2
    b = (np.asarray(ref, np.float64) + 1) / 2
    return 10 * math.log10(1.0 / np.mean((a - b) ** 2))


def batch(cfg, seed):
    """The synthetic (x, y) pair of a case (tests/test_golden_gpu.py builds the same)."""
    x, y = synthetic_pair(cfg["N"], cfg["H"], seed=seed)
    if cfg.get("gray"):
        x = np.repeat(x.mean(-1, keepdims=True), 3, -1).astype(np.float32)
        y = np.repeat(y.mean(-1, keepdims=True), 3, -1).astype(np.float32)
    if cfg["scale"] > 1:
        x = np.ascontiguousarray(x[:, ::cfg["scale"], ::cfg["scale"], :])
    return x, y


def digest(out, prefix, arrays, k=N_SAMPLE):
    for n, a in arrays.items():
        flat = np.asarray(a, np.float64).ravel()
        idx = sample_idx(prefix + n, flat.size, k)
        out[f"{prefix}{n}|idx"] = idx
        out[f"{prefix}{n}|val"] = flat[idx]
        out[f"{prefix}{n}|l2"] = np.float64(np.linalg.norm(flat))
        out[f"{prefix}{n}|maxabs"] = np.float64(np.abs(flat).max())


def vgg_weights(seed):
    from dgan.graph import init_graph_variables
    from dgan.zoo import vgg19_features
    return init_graph_variables(vgg19_features(1), seed)


def gen_pix2pix(cfg):
    out = {}
    st = O.P2PState(width=1, seed=cfg["seed"], drop_rate=0.5, drop_seed=cfg["drop_seed"], identity=True)
    PV = vgg_weights(cfg["seed"] + 7) if cfg["content"] else None
    if PV is None:
        st.w["content"] = 0.0
    meta = dict(cfg, gvars=[n for n, _ in st.gvars], dvars=[n for n, _ in st.dvars],
                wcrc_G=weights_crc(st.G, [n for n, _ in st.gvars]),
                wcrc_D=weights_crc(st.D, [n for n, _ in st.dvars]),
                wcrc_V=weights_crc(PV, sorted(PV)) if PV is not None else None)
    x, y = batch(cfg, cfg["batch_seeds"][0])
    ref = O.train_step(st, x, y, return_grads=True, apply=True, PV=PV)
    out["s1|losses"] = np.array(ref["losses"], np.float64)
    out["s1|psnr"] = np.float64(psnr(ref["gen"], y))
    digest(out, "s1|gen|", {"G(x)": ref["gen"]}, N_GEN_SAMPLE)
    out["s1|logits_real"] = ref["logits_real"].astype(np.float64)
    out["s1|logits_fake"] = ref["logits_fake"].astype(np.float64)
    digest(out, "s1|gG|", ref["gG"])
    digest(out, "s1|gD|", ref["gD"])
    for k, v in st.Gs.items():
        out[f"s1|bnG|{k}"] = np.asarray(v, np.float64)
    for k, v in st.Ds.items():
        out[f"s1|bnD|{k}"] = np.asarray(v, np.float64)
    x2, y2 = batch(cfg, cfg["batch_seeds"][1])
    ref2 = O.train_step(st, x2, y2, apply=True, PV=PV)
    out["s2|losses"] = np.array(ref2["losses"], np.float64)
    digest(out, "s2|pG|", st.G)
    digest(out, "s2|pD|", st.D)
    return meta, out


def gen_sr(cfg):
    from dgan import zoo
    from dgan.graph import init_graph_variables
    kind = cfg["kind"]
    if kind == "srgan":
        gg = zoo.srgan_generator(scale=cfg["scale"])
        dg = zoo.sr_discriminator(df=32)
    elif kind == "fsrgan":
        gg = zoo.fsrgan_generator(gf=32, n_blocks=6)
        dg = zoo.sr_discriminator(df=32)
    else:
        gg = zoo.autoencoder_generator()
        dg = zoo.sr_discriminator(df=32, name="Discriminator")
    PG = init_graph_variables(gg, cfg["seed"])
    PD = init_graph_variables(dg, cfg["seed"] + 1)
    PV = vgg_weights(cfg["seed"] + 7)
    st = S.SRState(kind, PG, PD, PV, scale=cfg["scale"], lr=cfg["lr"])
    meta = dict(cfg, wcrc_G=weights_crc(PG, [n for n, _ in gg.var_list()]),
                wcrc_D=weights_crc(PD, [n for n, _ in dg.var_list()]), wcrc_V=weights_crc(PV, sorted(PV)))
    out = {}
    x, y = batch(cfg, cfg["batch_seeds"][0])
    ref = S.train_step(st, x, y, apply=True)
    out["s1|losses"] = np.array(ref["losses"], np.float64)
    out["s1|psnr"] = np.float64(psnr(ref["gen"], y))
    digest(out, "s1|gen|", {"G(x)": ref["gen"]}, N_GEN_SAMPLE)
    digest(out, "s1|gG|", ref["gG"])
    digest(out, "s1|gD|", ref["gD"])
    for k in st.Gs.mean:
        out[f"s1|bnG|{k}/moving_mean"] = np.asarray(st.Gs.mean[k], np.float64)
        out[f"s1|bnG|{k}/moving_variance"] = np.asarray(st.Gs.var[k], np.float64)
    for k in st.Ds.mean:
        out[f"s1|bnD|{k}/moving_mean"] = np.asarray(st.Ds.mean[k], np.float64)
        out[f"s1|bnD|{k}/moving_variance"] = np.asarray(st.Ds.var[k], np.float64)
    x2, y2 = batch(cfg, cfg["batch_seeds"][1])
    ref2 = S.train_step(st, x2, y2, apply=True)
    out["s2|losses"] = np.array(ref2["losses"], np.float64)
    digest(out, "s2|pG|", st.PG)
    digest(out, "s2|pD|", st.PD)
    return meta, out


def main(names):
    os.makedirs(OUT, exist_ok=True)
    for name in names:
        cfg = CASES[name]
        t0 = time.time()
        meta, out = gen_pix2pix(cfg) if cfg["kind"] == "pix2pix" else gen_sr(cfg)
        meta["case"] = name
        meta["generator"] = "scripts/gen_golden.py"
        out["meta"] = np.array(json.dumps(meta))
        path = os.path.join(OUT, name + ".npz")
        np.savez_compressed(path, **out)
        print(f"{name}: {len(out)} arrays, {os.path.getsize(path) / 1024:.0f} KiB, {time.time() - t0:.0f} s; "
              f"losses s1 {np.round(out['s1|losses'], 6).tolist()}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or list(CASES))
