"""The step the bench times is the step the parity tests check.

The pix2pix step (train_pix2pix.py:33-71) runs on up to five streams (dgan/trainer.py): D's
parameter backward beside the G path, D's forward beside the VGG19 forward, D(fake)'s input
gradient beside the VGG19 backward, G's early Adam over the up blocks beside the down blocks'
backward, the target's VGG19 forward beside G's forward.  The one-stream step (every overlap off:
what the profiles and the per-layer tables run) launches the same kernels in one order, so the two
must end bit-identical -- a missing stream join would show here as a difference, not as drift
hidden under a tolerance.  And the captured HIP graph the bench replays must equal the eager
launches from the same state.
"""
import numpy as np
import pytest
import torch

gpu = pytest.mark.gpu


class Args:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _model(width=1):
    from pix2pix import Pix2Pix
    return Pix2Pix(Args(crop_size=256, retrain=0, width=width, seed=77, dropout_seed=3, identity_loss=1,
                        content_loss=1))


def _pair(N=2):
    from dataloader import synthetic_pair
    x, y = synthetic_pair(N, 256, 11)
    return torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()


@gpu
def test_overlapped_step_is_bit_identical_to_one_stream_step(monkeypatch):
    from dgan import trainer as T
    x, y = _pair()
    mA = _model()
    trA = mA.trainer(x.shape)
    assert trA.side is not None and trA.side2 is not None and trA.side3 is not None and trA.side4 is not None
    states = []
    # three steps: the first runs the target's VGG19 on the main stream (shared weight planes not yet
    # settled), the next two fork it; dropout on, identity and content on, Adam applied
    for _ in range(3):
        trA.step(x, y)
    states.append(T.snapshot(trA))
    monkeypatch.setattr(T, "OVERLAP", False)
    mB = _model()
    trB = mB.trainer(x.shape)
    assert trB.side is None and trB.side2 is None and trB.side3 is None and trB.side4 is None
    for _ in range(3):
        trB.step(x, y)
    states.append(T.snapshot(trB))
    torch.cuda.synchronize()
    assert all(torch.isfinite(t.float()).all() for t in states[0].values())
    bad = T.state_diff(*states)
    assert not bad, f"one-stream and overlapped steps differ in {bad}"


@gpu
def test_graph_replay_is_bit_identical_to_eager_step():
    """The bench's capture sequence (dgan.dist.CAPTURE_MODE, a side-stream warm-up step) on the
    five-stream step with early Adam, full width, bs2, content on: one eager step and one replay
    from the same snapshot end bit-identical, and a second replay continues the trajectory."""
    from dgan import trainer as T
    from dgan.dist import CAPTURE_MODE
    x, y = _pair()
    m = _model()
    tr = m.trainer(x.shape)
    assert tr.side3 is not None   # (early Adam: no data-parallel sync)
    for _ in range(2):
        tr.step(x, y)
    torch.cuda.synchronize()
    s0 = T.snapshot(tr)
    tr.step(x, y)
    e1 = T.snapshot(tr)
    tr.step(x, y)
    e2 = T.snapshot(tr)
    T.restore(tr, s0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        tr.step(x, y)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
        tr.step(x, y)
    torch.cuda.synchronize()
    T.restore(tr, s0)
    g.replay()
    r1 = T.snapshot(tr)
    g.replay()
    r2 = T.snapshot(tr)
    torch.cuda.synchronize()
    assert not T.state_diff(e1, r1), T.state_diff(e1, r1)
    assert not T.state_diff(e2, r2), T.state_diff(e2, r2)
    assert np.isfinite(r2["loss"].cpu().numpy()).all()
