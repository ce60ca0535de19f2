"""One network planned under different conv arithmetics, alternating.

The planner picks each op's GEMM arithmetic from its shape (csrc/conv.hip make_plan): the
frozen VGG19 of the content loss runs bf16x6 / fp32 tiles below X3_MIN_PIXELS and fp16x3 above
it (dgan/sr_trainer.py), the deep pix2pix layers fp32 tiles where their GEMM has few rows.  A
network's plans share its weight-operand planes; round 4 keyed that buffer by layer name
only, so a VGG19 planned at 32^2 (bf16x6, 6 B per weight), 64^2 (fp16x3 + bf16x6, 4 + 6 B) and
32^2 again wrote past the 6-B buffer (hipErrorIllegalAddress,
profiles/r4/x3_vgg64_fault_tests.log) or read the other format's planes.  The buffers are now
per (layer, plane format, bytes) and stamped with the weight version they were split from
(dgan/graph.py GraphPlan, ops.PlaneBuf).

Each call is checked against the fp64 oracle (mask-conditioned, as test_sr_gpu.py /
test_step_gpu.py) and bit for bit against a fresh network that only ever ran that one plan:
shared plane state that leaks between plans would move the result off the fresh network's.
Reference: /root/reference/pix2pix.py:45-67 (VGG19 content loss), train_pix2pix.py:51, :105
(the generator called at training and inference shapes)."""
import numpy as np
import pytest
import torch

from oracle import p2p_oracle as O
from oracle import sr_oracle as S


def _vsrc(cl):
    """(plan, slot, rows) of G(x)'s and of the target's VGG19 activations (ContentLoss)."""
    (pg, rg), (pt, rt) = cl.feature_sources()
    return (pg, 0, rg), (pt, 0, rt)

gpu = pytest.mark.gpu
DEV = "cuda"


def _vgg(seed, weights=None):
    from dgan.sr_trainer import VGGNetwork
    v = VGGNetwork(seed=seed)
    v.X3_MIN_PIXELS = 64 * 64   # fp16x3 from 64^2: 32^2 plans bf16x6 / fp32 tiles, 64^2 fp16x3
    if weights is not None:
        v.arena.load(weights)
    return v


def _content(vgg, gen, y):
    from dgan import ops
    from dgan.sr_trainer import ContentLoss
    N, H = gen.shape[0], gen.shape[1]
    key = ("cl", N, H)
    cl = vgg.__dict__.setdefault("_test_cl", {}).get(key)
    if cl is None:
        cl = vgg._test_cl[key] = ContentLoss(vgg, N, H, H, torch.device(DEV))
    ws = ops.Workspace()
    ws.get(cl.ws_bytes)
    dg = torch.zeros((N, H, H, 3), device=DEV)
    v = cl.forward(torch.from_numpy(gen).to(DEV), torch.from_numpy(y).to(DEV), ws=ws)
    cl.backward(dg, beta=0.0, ws=ws)
    torch.cuda.synchronize()
    return cl, v[0].item(), dg.cpu().numpy()


def _inputs(N, H, seed):
    from dataloader import synthetic_pair
    _, y = synthetic_pair(N, H, seed=seed)
    gen = np.tanh(np.arctanh(np.clip(y, -0.99, 0.99)) + 0.3 * np.random.default_rng(seed).standard_normal(y.shape))
    return gen.astype(np.float32), y


def _arith(cl, layer="block2_conv1"):
    p = cl.fplan
    for n in p.g.nodes:
        if n.kind == "conv" and n.name == layer:
            return p.desc[n.idx].op_arith("fwd"), cl.bplan.desc[n.idx].op_arith("bwd_data")
    raise KeyError(layer)


@gpu
@pytest.mark.timeout(600)
def test_vgg19_planned_across_arithmetics_alternating():
    """32^2 (bf16x6) -> 64^2 (fp16x3) -> 32^2 -> 64^2 at another batch -> new weights (arena.load)
    -> 32^2 -> 64^2: every call equals a fresh network's bit for bit and the fp64 oracle to the
    content test's bar (1e-5 of the gradient scale, test_sr_gpu.py)."""
    from gpu_decisions import audit_ok, graph_decisions, to_oracle
    vgg = _vgg(11)
    w0 = vgg.arena.export()
    w1 = {k: (v * 1.25).astype(np.float32) for k, v in w0.items()}
    seq = [(2, 32, w0), (2, 64, w0), (2, 32, w0), (1, 64, w0), (2, 64, w1), (2, 32, w1), (2, 64, w1)]
    ariths = {}
    cur = w0
    for step, (N, H, w) in enumerate(seq):
        if w is not cur:
            vgg.arena.load(w)   # (a frozen network's planes are stamped with the weight version)
            cur = w
        gen, y = _inputs(N, H, seed=3 + step)
        cl, val, dg = _content(vgg, gen, y)
        ariths[H] = _arith(cl)
        fresh = _vgg(11, w)
        _, val_f, dg_f = _content(fresh, gen, y)
        assert val == val_f, (step, N, H, val, val_f)
        assert np.array_equal(dg, dg_f), (step, N, H, float(np.abs(dg - dg_f).max()))
        PV = {k: torch.tensor(v.astype(np.float64)) for k, v in w.items()}
        dec = {"Vsr": to_oracle(graph_decisions(*_vsrc(cl)[0])),
               "Vhr": to_oracle(graph_decisions(*_vsrc(cl)[1]))}
        gt = torch.tensor(gen.astype(np.float64), requires_grad=True)
        c = S.content_loss(PV, torch.tensor(y.astype(np.float64)), gt, dec["Vsr"], dec["Vhr"])
        d0 = torch.autograd.grad(c, gt)[0].numpy()
        audit_ok(dec, 1e-5, f"content step {step} {N}x{H}")
        assert abs(val - c.item()) <= 2e-6 * abs(c.item()), (step, val, c.item())
        err = np.abs(dg - d0).max()
        assert err <= 1e-5 * np.abs(d0).max(), (step, N, H, err, np.abs(d0).max())
    # the sequence really alternates arithmetics (else it tests nothing)
    assert ariths[32] != ariths[64], ariths
    assert "f16x3" in ariths[64], ariths


class _Args:
    def __init__(self, **kw):
        self.crop_size = 256
        self.retrain = 0
        self.content_loss = 0
        self.__dict__.update(kw)


@gpu
@pytest.mark.timeout(600)
def test_pix2pix_networks_planned_at_several_shapes_alternating():
    """The pix2pix G and D planned for training over 2N images (both halves in one pass), for
    the N-image G-path backward through D(fake), and for inference at N = 1, 2 and at 512^2,
    alternating: losses of each training step (apply=False: the weights stay) against the fp64
    oracle and bit for bit against a fresh model, inference outputs against the fp64 oracle's
    moving-statistics forward and bit for bit against a fresh model."""
    from pix2pix import Pix2Pix
    width, seed = 4, 23

    def model():
        return Pix2Pix(_Args(width=width, seed=seed, dropout_seed=2, dropout_rate=0.5))

    m = model()
    G0, D0 = m.generator.arena.export(), m.discriminator.arena.export()
    xs = {n: O.synthetic_pair(n, 256, seed=40 + n) for n in (1, 2, 3)}
    xl, _ = O.synthetic_pair(1, 512, seed=50)
    seq = [("train", 2), ("infer", 1), ("train", 3), ("infer", 2), ("train", 2), ("infer512", 1), ("train", 3)]
    for step, (what, n) in enumerate(seq):
        if what == "train":
            x, y = xs[n]
            loss = m.trainer(x.shape).step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), apply=False)
            torch.cuda.synchronize()
            got = loss.cpu().numpy()
            st = O.P2PState(width=width, seed=seed, drop_rate=0.5, drop_seed=2)
            st.G = {k: v.copy() for k, v in G0.items()}
            st.D = {k: v.copy() for k, v in D0.items()}
            ref = O.train_step(st, x, y, apply=False)
            assert np.allclose(got.astype(np.float64), np.array(ref["losses"]), rtol=1e-5, atol=1e-7), (step, got)
            f = model()
            want = f.trainer(x.shape).step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(),
                                           apply=False).cpu().numpy()
            assert np.array_equal(got, want), (step, what, n, got, want)
        else:
            x = xs[n][0] if what == "infer" else xl
            out = m.generator(x, training=False).cpu().numpy()
            states = m.generator.bn.export()
            ref, _ = O.generator_forward(G0, x, width, training=False, states=states)
            assert np.abs(out - ref).max() < 1e-5, (step, what, float(np.abs(out - ref).max()))
            f = model()
            f.generator.bn.load(states)
            want = f.generator(x, training=False).cpu().numpy()
            assert np.array_equal(out, want), (step, what, n)

    # the sequence really alternates arithmetics, not only shapes: at width 4
    # the 2N = 4 and 2N = 6 training plans run G up5 / up6 in different arithmetics (fp32 tiles at
    # 4 images, fp16x3 at 6), so the alternation above switches plans of both kinds on one network
    def ariths(n):
        tr = m.trainer(xs[n][0].shape)
        return [(d.label, o, d.op_arith(o)) for d in tr.G.ddesc + tr.G.udesc + [tr.G.ldesc] + tr.D.desc
                for o in ("fwd", "bwd_data", "bwd_filter")]
    a2, a3 = ariths(2), ariths(3)
    moved = [(l, o, p, q) for (l, o, p), (_, _, q) in zip(a2, a3) if p != q]
    assert moved, "the alternating training plans run every op in one arithmetic"
    assert any(q == "f16x3" for *_, q in moved) and any(p == "fp32" for *_, p, _ in moved), moved
