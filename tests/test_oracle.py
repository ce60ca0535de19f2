"""The CPU oracle itself: known-answer tests of each TF/Keras semantic it
restates (oracle/p2p_oracle.py header, items 1-9), the reference's layer
bookkeeping, and agreement of its hand-written backward with an independent
torch fp64 autograd restatement of the same graph (oracle/torch_p2p.py)."""
import numpy as np
import pytest
import torch

from oracle import p2p_oracle as O
from oracle import torch_p2p as T


def test_tf_same_padding_known_answers():
    # item 1: total = max((ceil(H/s)-1)*s + k - H, 0), before = total//2 (extra after)
    assert O.tf_same_pads(256, 4, 2) == (1, 1)     # pix2pix downsample
    assert O.tf_same_pads(6, 3, 2) == (0, 1)       # SRGAN/FSRGAN D k3 s2: asymmetric
    assert O.tf_same_pads(5, 3, 2) == (1, 1)
    assert O.tf_same_pads(7, 3, 1) == (1, 1)
    assert O.tf_same_pads(7, 4, 1) == (1, 2)
    assert O.tf_same_pads(7, 1, 1) == (0, 0)


def test_conv_transpose_is_adjoint_of_conv():
    # item 2: <convT(x), y> == <x, conv(y)>, output H*s
    rng = np.random.default_rng(0)
    x = rng.standard_normal((2, 5, 6, 4))
    w = rng.standard_normal((4, 4, 3, 4))  # [k,k,F,Cin]
    y = rng.standard_normal((2, 10, 12, 3))
    t = O.convT_fwd(x, w, 2)
    assert t.shape == (2, 10, 12, 3)
    lhs = (t * y).sum()
    rhs = (x * O.conv_fwd(y, w, 2, (1, 1, 1, 1))).sum()
    assert abs(lhs - rhs) < 1e-9 * abs(lhs)


def test_conv_matches_direct_loops():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((1, 5, 5, 2))
    w = rng.standard_normal((3, 3, 2, 2))
    pads = O.tf_same_pads(5, 3, 2) + O.tf_same_pads(5, 3, 2)
    y = O.conv_fwd(x, w, 2, pads)
    xp = np.pad(x, ((0, 0), (pads[0], pads[1]), (pads[2], pads[3]), (0, 0)))
    for ho in range(y.shape[1]):
        for wo in range(y.shape[2]):
            for co in range(2):
                ref = sum(xp[0, ho * 2 + i, wo * 2 + j, ci] * w[i, j, ci, co]
                          for i in range(3) for j in range(3) for ci in range(2))
                assert abs(y[0, ho, wo, co] - ref) < 1e-12


def test_activations_and_grads_at_zero():
    # item 3: LeakyReLU alpha 0.3, grad at 0 is alpha; ReLU grad at 0 is 0
    v = np.array([-2.0, 0.0, 3.0])
    assert np.allclose(O.lrelu(v), [-0.6, 0.0, 3.0])
    assert np.allclose(np.where(v > 0, 1.0, O.ALPHA), [0.3, 0.3, 1.0])


def test_batchnorm_known_answer():
    # item 4: biased variance, eps 1e-3; moving stats use the unbiased variance
    y = np.array([1.0, 2.0, 3.0, 4.0]).reshape(1, 2, 2, 1)
    b, c = O.bn_train(y, np.ones(1), np.zeros(1))
    assert np.isclose(c["mu"][0], 2.5) and np.isclose(c["var"][0], 1.25)
    assert np.allclose(b.ravel(), (np.array([1, 2, 3, 4]) - 2.5) / np.sqrt(1.25 + 1e-3))
    st = {"l/moving_mean": np.zeros(1, np.float32), "l/moving_variance": np.ones(1, np.float32)}
    O.bn_update_moving(st, "l", c)
    assert np.isclose(st["l/moving_mean"][0], 0.025)
    assert np.isclose(st["l/moving_variance"][0], 0.99 + 0.01 * (1.25 * 4 / 3), rtol=1e-6)


def test_bce_with_logits_known_answers():
    # item 5
    assert np.isclose(O.bce_logits(np.array(0.0), 1.0), np.log(2.0))
    assert np.isclose(O.bce_logits(np.array(2.0), 0.0), np.log1p(np.exp(2.0)))
    assert np.isclose(O.bce_logits(np.array(-30.0), 1.0), 30.0, rtol=1e-12)


def test_total_variation_known_answer():
    # item 6: per image sum |dh| + |dw| over all channels, mean over batch
    img = np.zeros((2, 2, 2, 1))
    img[0, 0, 0, 0] = 1.0
    vals, _ = O.losses_and_grads(gen=np.zeros_like(img), tgt=img, ident=None, zr=np.zeros(1), zf=np.zeros(1),
                                 w=dict(O.LOSS_WEIGHTS, tv=1.0))
    assert np.isclose(vals[6], (1.0 + 1.0) / 2)


def test_mean_losses_and_sign_at_zero():
    # item 7
    t = np.array([0.5, -0.5, 0.0, 0.25]).reshape(1, 1, 4, 1)
    g = np.array([0.0, 0.0, 0.0, 0.25]).reshape(1, 1, 4, 1)
    vals, gr = O.losses_and_grads(g, t, None, np.zeros(1), np.zeros(1), w=dict(O.LOSS_WEIGHTS, tv=0.0))
    assert np.isclose(vals[2], 0.25) and np.isclose(vals[3], 0.125)
    # entries with d == 0 get no L1 gradient
    dl1 = -(np.sign(t - g) / 4)
    assert dl1.ravel()[2] == 0 and dl1.ravel()[3] == 0


def test_keras_adam_first_step():
    # item 8: first step moves each parameter by ~lr (epsilon on sqrt(v))
    p = np.array([1.0, 1.0], np.float32)
    g = np.array([0.3, -5.0])
    p1, m, v = O.adam_update(p, g, np.zeros(2, np.float32), np.zeros(2, np.float32), t=1)
    assert np.allclose(p.astype(np.float64) - p1, 2e-4 * np.sign(g), rtol=2e-3)
    # epsilon placement: with g tiny the update is g*sqrt(1-b2)/(|g|sqrt(1-b2)+eps)*lr, not lr
    p2, _, _ = O.adam_update(p, np.array([1e-7, 1e-7]), np.zeros(2, np.float32), np.zeros(2, np.float32), t=1)
    expect = 2e-4 * (1e-7 * np.sqrt(1e-3)) / (1e-7 * np.sqrt(1e-3) + 1e-7)
    assert np.allclose(p - p2, expect, rtol=1e-3)


def test_variable_counts_match_reference_model():
    # G 54,414,979 and D 2,768,641 trainable parameters (pix2pix.py:144-220)
    ng = sum(int(np.prod(s)) for _, s in O.g_variables())
    nd = sum(int(np.prod(s)) for _, s in O.d_variables())
    assert ng == 54_414_979
    assert nd == 2_768_641


def test_dropout_hash_properties():
    m1 = O.dropout_mask(123, 5, 100000, 0.5)
    m2 = O.dropout_mask(123, 5, 100000, 0.5)
    m3 = O.dropout_mask(123, 6, 100000, 0.5)
    assert np.array_equal(m1, m2)
    assert not np.array_equal(m1, m3)
    assert abs(m1.mean() - 0.5) < 0.01
    assert O.dropout_mask(1, 0, 1000, 0.0).all()


def test_synthetic_pair_range():
    x, y = O.synthetic_pair(2, 64, seed=0)
    assert x.shape == y.shape == (2, 64, 64, 3)
    assert x.dtype == np.float32
    assert -1 <= x.min() and x.max() <= 1 and -1 <= y.min() and y.max() <= 1
    assert 0.05 < np.abs(x - y).mean() < 0.1


@pytest.mark.parametrize("drop_rate", [0.0, 0.5])
def test_oracle_backward_matches_torch_autograd(drop_rate):
    """Tiny-width pix2pix (filters/16) at the full 256x256 spatial size, bs2."""
    width = 16
    st = O.P2PState(width=width, seed=3, drop_rate=drop_rate, drop_seed=11)
    x, y = O.synthetic_pair(2, 256, seed=5)
    out = O.train_step(st, x, y, return_grads=True, apply=False)
    vals, gG, gD, gen = T.step_grads(st.G, st.D, x, y, width, drop_rate, st.drop_seed, 0)
    assert np.allclose(out["gen"], gen, rtol=0, atol=1e-12)
    assert np.allclose(np.array(out["losses"]), np.array(vals), rtol=1e-10, atol=1e-14)
    for k in gG:
        ref = gG[k]
        err = np.abs(out["gG"][k] - ref).max()
        assert err <= 1e-9 * (np.abs(ref).max() + 1e-12), (k, err)
    for k in gD:
        ref = gD[k]
        err = np.abs(out["gD"][k] - ref).max()
        assert err <= 1e-9 * (np.abs(ref).max() + 1e-12), (k, err)
