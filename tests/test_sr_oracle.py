"""Known-answer tests of the TF semantics the SR-family oracle restates
(oracle/sr_oracle.py S1-S7), and structural agreement between the product's
network graphs (dgan.zoo) and the oracle's independent restatements of
srgan.py / fsrgan.py / autoencoder.py / VGG19.  CPU only."""
import math

import numpy as np
import pytest
import torch

from oracle import sr_oracle as S


def test_prelu_matches_keras_definition():
    x = torch.tensor([[[[-2.0, 3.0], [0.0, -0.5]]]], dtype=torch.float64)   # [1,1,2,2]
    a = torch.tensor([[[0.25, -1.0]]], dtype=torch.float64)
    y = S.prelu(x, a)
    # relu(x) - alpha * relu(-x)
    assert y.tolist() == [[[[-0.5, 3.0], [0.0, 0.5]]]]


def test_depth_to_space_dcr_order():
    # TF doc example: input [1,1,1,4] -> [1,2,2,1] in (i*2+j) order
    x = torch.arange(4, dtype=torch.float64).reshape(1, 1, 1, 4)
    y = S.depth_to_space(x, 2)
    assert y.shape == (1, 2, 2, 1)
    assert y[0, :, :, 0].tolist() == [[0.0, 1.0], [2.0, 3.0]]
    # with 2 output channels: in[..., (i*2+j)*C + c]
    x = torch.arange(8, dtype=torch.float64).reshape(1, 1, 1, 8)
    y = S.depth_to_space(x, 2)
    assert y[0, 1, 0].tolist() == [4.0, 5.0]


def test_depthwise_conv_is_per_channel_correlation():
    rng = np.random.default_rng(0)
    x = torch.tensor(rng.standard_normal((1, 5, 4, 3)))
    k = torch.tensor(rng.standard_normal((3, 3, 3, 1)))
    b = torch.tensor(rng.standard_normal(3))
    y = S.dwconv3(x, k, b)
    xp = np.pad(x.numpy(), ((0, 0), (1, 1), (1, 1), (0, 0)))
    ref = np.zeros((1, 5, 4, 3))
    for h in range(5):
        for w in range(4):
            for c in range(3):
                ref[0, h, w, c] = b[c].item() + sum(xp[0, h + i, w + j, c] * k[i, j, c, 0].item()
                                                    for i in range(3) for j in range(3))
    assert np.allclose(y.numpy(), ref, atol=1e-12)


def test_maxpool_and_nearest_upsample():
    x = torch.arange(16, dtype=torch.float64).reshape(1, 4, 4, 1)
    assert S.maxpool2(x)[0, :, :, 0].tolist() == [[5.0, 7.0], [13.0, 15.0]]
    # 'valid' floor for odd sizes (VGG19 on 24x24 -> 3x3 -> 1x1)
    assert S.maxpool2(torch.zeros(1, 3, 3, 2, dtype=torch.float64)).shape == (1, 1, 1, 2)
    u = S.upsample2(torch.tensor([[[[1.0], [2.0]]]], dtype=torch.float64))
    assert u[0, :, :, 0].tolist() == [[1.0, 1.0, 2.0, 2.0], [1.0, 1.0, 2.0, 2.0]]


def test_vgg_preprocess_caffe():
    img = torch.tensor([[[[-1.0, 0.0, 1.0]]]], dtype=torch.float64)  # RGB
    z = S.vgg_preprocess(img)
    # -> pixel (0, 127.5, 255) RGB -> BGR (255, 127.5, 0) minus caffe means
    assert np.allclose(z.numpy().ravel(), [255 - 103.939, 127.5 - 116.779, 0 - 123.68])


def test_bce_on_sigmoid_equals_logit_bce():
    z = torch.tensor([-3.0, 0.0, 2.5], dtype=torch.float64)
    p = torch.sigmoid(z)
    for y in (0.0, 1.0):
        prob = -(y * torch.log(p) + (1 - y) * torch.log(1 - p)).mean()
        assert abs(prob.item() - S.bce_logits(z, y).item()) < 1e-12


def test_exponential_decay_staircase():
    assert S.exp_decay(1e-3, 0) == 1e-3
    assert S.exp_decay(1e-3, 99999) == 1e-3
    assert abs(S.exp_decay(1e-3, 100000) - 1e-4) < 1e-18
    assert abs(S.exp_decay(1e-3, 250000) - 1e-5) < 1e-18
    assert abs(S.exp_decay(1e-3, 50000, staircase=False) - 1e-3 * 0.1 ** 0.5) < 1e-15


def test_total_variation_per_image():
    img = torch.zeros(2, 2, 2, 1, dtype=torch.float64)
    img[0, 0, 0, 0] = 1.0
    tv = S.total_variation(img)
    assert tv.tolist() == [2.0, 0.0]


# -------------------------------------------------------------------------
# product graphs vs oracle restatements (names, shapes, forward on CPU)
# -------------------------------------------------------------------------
def _graph_weights(graph, seed=3):
    from dgan.graph import init_graph_variables
    return {k: torch.tensor(v.astype(np.float64)) for k, v in init_graph_variables(graph, seed).items()}


def test_srgan_graph_matches_oracle_variables_and_forward():
    from dgan import zoo
    g = zoo.srgan_generator(scale=4)
    P = _graph_weights(g)
    x = torch.tensor(np.random.default_rng(1).uniform(-1, 1, (1, 6, 6, 3)))
    out = S.srgan_generator(P, x, S.BNStats(), scale=4)
    assert out.shape == (1, 24, 24, 3)
    d = zoo.sr_discriminator()
    z = S.sr_discriminator(_graph_weights(d), out, S.BNStats())
    assert z.shape == (1, 2, 2, 1)
    # every product variable is read by the oracle (no dead or misnamed layers)
    n_gen = sum(int(np.prod(s)) for _, s in g.var_list())
    assert n_gen == 1728 + 128 + 64 + 16 * (2 * 36864 + 2 * 128) + 36864 + 128 + 2 * (147456 + 256 + 64) + 195


def test_fsrgan_graph_matches_oracle():
    from dgan import zoo
    g = zoo.fsrgan_generator()
    x = torch.tensor(np.random.default_rng(2).uniform(-1, 1, (1, 8, 8, 3)))
    out = S.fsrgan_generator(_graph_weights(g), x, S.BNStats())
    assert out.shape == (1, 32, 32, 3)
    names = {n for n, _ in g.var_list()}
    assert "expanded_conv_depthwise/depthwise_kernel" in names and "block_5_project_BN/gamma" in names
    assert "block_0_expand/kernel" not in names  # block 0 has no expansion (fsrgan.py:140-151)


def test_autoencoder_graph_matches_oracle():
    from dgan import zoo
    g = zoo.autoencoder_generator()
    x = torch.tensor(np.random.default_rng(3).uniform(-1, 1, (1, 32, 32, 3)))
    out = S.autoencoder_generator(_graph_weights(g), x)
    assert out.shape == (1, 32, 32, 3)
    shapes = dict(g.var_list())
    assert shapes["conv6/kernel"] == (3, 3, 176, 152)   # concat(up(pool5) 100, pool4 76)
    assert shapes["conv10/kernel"] == (3, 3, 67, 64)    # concat(up(conv9b) 64, input 3)


def test_vgg_graph_matches_oracle():
    from dgan import zoo
    g = zoo.vgg19_features(width=8)
    x = torch.tensor(np.random.default_rng(4).uniform(-100, 100, (1, 32, 32, 3)))
    f = S.vgg19(_graph_weights(g), x)
    assert f.shape == (1, 2, 2, 64)
    full = zoo.vgg19_features()
    n = sum(int(np.prod(s)) for _, s in full.var_list())
    assert n == 20024384   # keras VGG19(include_top=False) up to block5_conv4 (block5_conv4 incl.)


def test_graph_plan_beta_schedule_on_cpu_shapes():
    """Gradient fan-in bookkeeping: a residual skip input is written once with
    beta 0 and accumulated after; concat members alias the concat buffer."""
    from dgan import zoo
    from dgan.graph import Graph
    g = Graph("t")
    a = g.conv(g.input, 8, 3, name="c1")
    b = g.conv(a, 8, 3, name="c2")
    s = g.add(a, b, name="s")
    g.set_output(g.conv(s, 3, 1, name="c3"))
    cons = g.consumers()
    assert [n.name for n in cons[a.id]] == ["c2", "s"]
    ae = zoo.autoencoder_generator()
    kinds = [n.kind for n in ae.nodes]
    assert kinds.count("concat") == 5 and kinds.count("maxpool") == 5 and kinds.count("upsample") == 5


def test_decisions_plain_and_forced():
    """oracle/decisions.py: forcing the oracle's own decisions changes nothing; forcing a flipped
    decision on a clear (non-tie) value is reported by the audit."""
    import torch
    from oracle.decisions import Decisions
    rng = np.random.default_rng(4)
    x = torch.tensor(rng.standard_normal((2, 4, 6, 5)), requires_grad=True)
    a = torch.tensor([0.2] * 5)
    plain = Decisions()
    own = {"r": (x > 0).detach().numpy(), "p": torch.tensor(rng.standard_normal((2, 4, 6, 5))).numpy()}
    win = x.detach().reshape(2, 2, 2, 3, 2, 5).permute(0, 1, 3, 5, 2, 4).reshape(2, 2, 3, 5, 4)
    own["p"] = win.argmax(-1).numpy()
    forced = Decisions(own | {"l": own["r"], "q": own["r"]})
    for d in (plain, forced):
        y = d.relu("r", x).sum() + d.lrelu("l", x, 0.3).sum() + d.prelu("q", x, a).sum() + d.maxpool2("p", x).sum()
        g = torch.autograd.grad(y, x)[0]
        if d is plain:
            y0, g0 = y.detach(), g
    assert torch.equal(y.detach(), y0) and torch.equal(g, g0)
    assert forced.worst()[0] == 0
    flip = own["r"].copy()
    i = np.unravel_index(np.argmax(np.abs(x.detach().numpy())), flip.shape)
    flip[i] = ~flip[i]
    d = Decisions({"r": flip})
    d.relu("r", x)
    n, worst, where = d.worst()
    assert n == 1 and worst == 1.0 and where == "r"
