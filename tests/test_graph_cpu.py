"""Host-side graph-executor decisions (dgan/graph.py), planned on the CPU (no kernel runs:
descriptors plan at creation, buffers are host tensors).

The BN + residual Add fusion and the Add gradient sharing of the SR family's residual
blocks (srgan.py:165-181, fsrgan.py:176-214): which BNs write their Add's output, which
Add inputs share the Add's gradient buffer, and the ordering invariant that makes the
sharing exact -- every other writer of a shared input gradient runs (in backward order)
after every reader of the Add's gradient.  The GPU test
`test_bn_residual_add_fusion_is_bit_identical` holds the fused step to the unfused one
bit for bit."""
import pytest
import torch

from test_fp16_gpu import Args


@pytest.fixture
def cpu_models(monkeypatch):
    from dgan import models, sr_models
    monkeypatch.setattr(models, "default_device", lambda: torch.device("cpu"))
    monkeypatch.setattr(sr_models, "default_device", lambda: torch.device("cpu"))
    monkeypatch.delenv("DG_NO_BN_ADD", raising=False)
    monkeypatch.delenv("DG_NO_ADD_ALIAS", raising=False)


def _generator_plan(which):
    if which == "srgan":
        from srgan import SRGAN as cls
    else:
        from fsrgan import FastSRGAN as cls
    m = cls(Args(crop_size=32))
    return m.generator.plan(2, 8, 8, slots=1, train=True)


@pytest.mark.parametrize("which", ["srgan", "fsrgan"])
def test_bn_add_fusion_decisions(which, cpu_models):
    p = _generator_plan(which)
    nodes = p.g.nodes
    cons = {}
    for n in nodes[1:]:
        for t in n.ins:
            cons.setdefault(t.id, []).append(n)
    assert p.bn_add, "no BN + Add fused"
    for b, (a, skip) in p.bn_add.items():
        bn = nodes[b]
        assert bn.kind == "bn" and a.kind == "add" and bn.attrs["act"] in ("none", "linear", None)
        assert cons[bn.out.id] == [a] and skip.id != bn.out.id
        # the BN's output gradient IS the Add's
        assert p.grad[bn.out.id] is p.grad[a.out.id]
    shared = 0
    for ai, al in p.add_alias.items():
        a = nodes[ai]
        bn = p.add_of_bn.get(ai)
        lim = bn.idx if bn is not None else ai
        for tid in al:
            assert p.grad[tid] is p.grad[a.out.id]
            if bn is not None and tid == bn.out.id:
                continue
            shared += 1
            # the Add writes this gradient first (beta 0) and every other consumer of the
            # skip input runs after the BN / Add backward has read the shared buffer
            assert p.beta[(ai, tid)] == 0.0
            assert all(c.idx < lim for c in cons[tid] if c is not a), (a.name, tid)
    if which == "srgan":
        # 16 residual blocks + the long skip: 17 BNs fused, 16 skip inputs shared (every
        # block input but the first, which the long skip's Add writes first)
        assert len(p.bn_add) == 17 and shared == 16
    else:
        assert shared >= 1


def test_bn_add_switches(cpu_models, monkeypatch):
    monkeypatch.setenv("DG_NO_BN_ADD", "1")
    p = _generator_plan("srgan")
    # unfused: each Add still shares its gradient with one input (the BN output, which
    # only it consumes)
    assert not p.bn_add and sum(len(v) for v in p.add_alias.values()) == 17
    monkeypatch.setenv("DG_NO_ADD_ALIAS", "1")
    p = _generator_plan("srgan")
    assert not p.bn_add and not any(p.add_alias.values())


def test_bn_add_not_fused_when_skip_is_produced_later(cpu_models):
    """A linear BN feeding an Add whose other input is computed AFTER the BN (in node
    order) must not be fused: the fused BN would read the skip before it is written."""
    from dgan.graph import Graph, GraphNetwork
    g = Graph("late_skip")
    a = g.conv(g.input, 8, 3, name="a")
    b = g.bn(a, name="b")                      # linear BN, only consumer: the Add
    late = g.conv(g.input, 8, 3, name="late")  # the skip, produced after the BN
    g.set_output(g.conv(g.add(b, late, name="add"), 3, 3, name="out"))
    p = GraphNetwork(g, seed=1, device=torch.device("cpu")).plan(2, 8, 8, slots=1, train=True)
    assert not p.bn_add

    g2 = Graph("early_skip")
    early = g2.conv(g2.input, 8, 3, name="early")
    b2 = g2.bn(g2.conv(g2.input, 8, 3, name="a"), name="b")
    g2.set_output(g2.conv(g2.add(b2, early, name="add"), 3, 3, name="out"))
    p2 = GraphNetwork(g2, seed=1, device=torch.device("cpu")).plan(2, 8, 8, slots=1, train=True)
    assert len(p2.bn_add) == 1
