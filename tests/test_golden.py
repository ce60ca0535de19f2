"""The committed golden fixtures (tests/golden/, scripts/gen_golden.py) on the
CPU: they load with the safe loader, the product's seeded initialisers still
produce the weights they were generated from (crc32 per network), and the
fp64 oracle still reproduces the small case's first step."""
import numpy as np
import pytest

from golden_util import batch, load, weights_crc

CASES = ["p2p_bs16", "p2p_bs16_core", "srgan_bs32", "ae_bs4", "fsrgan_bs8"]


@pytest.mark.parametrize("case", CASES)
def test_fixture_loads_and_weights_match(case):
    from dgan import zoo
    from dgan.graph import init_graph_variables
    meta, d = load(case)
    assert meta["case"] == case
    assert np.isfinite(d["s1|losses"]).all() and np.isfinite(d["s2|losses"]).all()
    if meta["kind"] == "pix2pix":
        from dgan.nets import d_variables, g_variables, init_variables
        G = init_variables(g_variables(1), meta["seed"])
        D = init_variables(d_variables(1), meta["seed"] + 1)
        assert weights_crc(G, meta["gvars"]) == meta["wcrc_G"]
        assert weights_crc(D, meta["dvars"]) == meta["wcrc_D"]
    else:
        gg = {"srgan": lambda: zoo.srgan_generator(scale=meta["scale"]),
              "fsrgan": lambda: zoo.fsrgan_generator(gf=32, n_blocks=6)}.get(meta["kind"], zoo.autoencoder_generator)()
        dg = zoo.sr_discriminator(df=32)
        G = init_graph_variables(gg, meta["seed"])
        D = init_graph_variables(dg, meta["seed"] + 1)
        assert weights_crc(G, [n for n, _ in gg.var_list()]) == meta["wcrc_G"]
        assert weights_crc(D, [n for n, _ in dg.var_list()]) == meta["wcrc_D"]
    if meta.get("content", 1):
        V = init_graph_variables(zoo.vgg19_features(1), meta["seed"] + 7)
        assert weights_crc(V, sorted(V)) == meta["wcrc_V"]
    x, y = batch(meta, meta["batch_seeds"][0])
    assert x.shape[0] == meta["N"] and y.shape[1] == meta["H"]
    assert x.min() >= -1 and x.max() <= 1


def test_oracle_reproduces_ae_fixture():
    """oracle/sr_oracle.py re-run on the ae_bs4 config reproduces the committed step-1 losses and
    gradients (pins the oracle against drift once the fixtures exist)."""
    from dgan import zoo
    from dgan.graph import init_graph_variables
    from oracle import sr_oracle as S
    from golden_util import compare_digest
    meta, d = load("ae_bs4")
    PG = init_graph_variables(zoo.autoencoder_generator(), meta["seed"])
    PD = init_graph_variables(zoo.sr_discriminator(df=32, name="Discriminator"), meta["seed"] + 1)
    PV = init_graph_variables(zoo.vgg19_features(1), meta["seed"] + 7)
    st = S.SRState("autoencoder", PG, PD, PV, scale=1, lr=meta["lr"])
    x, y = batch(meta, meta["batch_seeds"][0])
    ref = S.train_step(st, x, y, apply=False)
    assert np.allclose(ref["losses"], d["s1|losses"], rtol=1e-9, atol=1e-12)
    compare_digest(d, "s1|gG|", ref["gG"], 1e-10, what="G")
    compare_digest(d, "s1|gD|", ref["gD"], 1e-10, what="D")
