"""The reference-driver surface on the HIP path (train_pix2pix.py:33-195,
pix2pix.py:74-103): the functions a user's scripts call, checked against the
fused trainer they wrap, the oracle, and an uninterrupted run.

  train_step(model, x, y)              8-tuple == the trainer's loss vector, same weights after
  Pix2Pix.generator_loss / discriminator_loss   values vs oracle/p2p_oracle.py
  Adam.apply_gradients(zip(g, trainable_variables))   bit-equal to one arena-wide dg_adam
  main(args): 2 epochs  ==  1 epoch, checkpoint, restore (--retrain), 1 epoch   (bit-identical)
"""
import numpy as np
import pytest
import torch

from oracle import p2p_oracle as O

gpu = pytest.mark.gpu


class Args:
    def __init__(self, **kw):
        self.crop_size = 256
        self.retrain = 0
        self.width = 16
        self.seed = 9
        self.dropout_seed = 2
        self.content_loss = 0
        self.__dict__.update(kw)


@gpu
def test_train_step_tuple_equals_trainer():
    import train_pix2pix
    from pix2pix import Pix2Pix
    x, y = O.synthetic_pair(2, 256, seed=4)
    a, b = Pix2Pix(Args()), Pix2Pix(Args())
    out = train_pix2pix.train_step(a, x, y)           # numpy in, device scalars out
    assert len(out) == 8 and all(t.dim() == 0 for t in out)
    ref = b.trainer(x.shape).step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
    torch.cuda.synchronize()
    assert torch.equal(torch.stack(out), ref)
    assert torch.equal(a.generator.arena.data, b.generator.arena.data)
    assert torch.equal(a.discriminator.arena.data, b.discriminator.arena.data)
    assert a.gen_optimizer.iterations == 1 and a.disc_optimizer.iterations == 1


@gpu
def test_generator_and_discriminator_loss_match_oracle():
    """generator_loss (pix2pix.py:74-94, identity pass G(target) inside) and
    discriminator_loss (:96-103) on the GPU's own G / D outputs."""
    from pix2pix import Pix2Pix
    m = Pix2Pix(Args(dropout_rate=0.0))
    x, y = O.synthetic_pair(2, 256, seed=6)
    gen = m.generator(x, training=True)
    zr = m.discriminator([x, y], training=True)
    zf = m.discriminator([x, gen], training=True)
    g7 = m.generator_loss(zf, gen, y)
    ident = m.generator(y, training=True)             # what generator_loss ran internally
    disc = m.discriminator_loss(zr, zf)
    torch.cuda.synchronize()
    h = lambda t: t.detach().cpu().numpy().astype(np.float64)
    vals, _ = O.losses_and_grads(h(gen), y, h(ident), h(zr), h(zf))
    total, gan, l1, l2, cont, dsc, var, idl = vals
    got = [float(t) for t in g7]
    assert len(g7) == 7
    assert np.allclose(got, [total, gan, l1, l2, cont, var, idl], rtol=2e-6, atol=1e-8), (got, vals)
    assert np.isclose(float(disc), dsc, rtol=2e-6)


@gpu
def test_adam_apply_gradients_equals_arena_adam():
    from dgan import ops
    from pix2pix import Pix2Pix
    x, y = O.synthetic_pair(2, 256, seed=8)
    a, b = Pix2Pix(Args()), Pix2Pix(Args())
    a.trainer(x.shape).step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), apply=False)
    for net_a, net_b, opt in ((a.generator, b.generator, a.gen_optimizer),
                              (a.discriminator, b.discriminator, a.disc_optimizer)):
        A, B = net_a.arena, net_b.arena
        B.grad.copy_(A.grad)
        grads = [A.grad_of(n) for n, _ in A.var_list]
        opt.apply_gradients(zip(grads, net_a.trainable_variables))
        ops.adam(B.data, B.grad, B.m, B.v, 2e-4, 0.5, 0.999, 1e-7, B.iterations)
        ops.counter_add(B.iterations, 1)
    torch.cuda.synchronize()
    for na, nb in ((a.generator, b.generator), (a.discriminator, b.discriminator)):
        assert torch.equal(na.arena.data, nb.arena.data)
        assert torch.equal(na.arena.m, nb.arena.m) and torch.equal(na.arena.v, nb.arena.v)
        assert int(na.arena.iterations.item()) == 1


def _main_args(tmp, epochs, retrain):
    import train_pix2pix
    a = train_pix2pix.parse_args([])
    a.model_dir, a.logdir = str(tmp / "models"), str(tmp / "logs")
    a.batch_size, a.epochs, a.retrain, a.synthetic, a.steps_per_epoch = 2, epochs, retrain, 1, 2
    a.save_iter = 2
    a.width, a.seed, a.content_loss, a.dropout_seed = 16, 5, 0, 1
    return a


@gpu
def test_main_checkpoint_resume_is_bit_identical(tmp_path):
    """main() for 2 epochs vs main() 1 epoch + restore (--retrain 1) + 1 epoch: the same
    weights, Adam slots, BN statistics, counters (train_pix2pix.py:156-195)."""
    import train_pix2pix
    full = train_pix2pix.main(_main_args(tmp_path / "a", 2, 0))
    train_pix2pix.main(_main_args(tmp_path / "b", 1, 0))
    resumed = train_pix2pix.main(_main_args(tmp_path / "b", 1, 1))
    torch.cuda.synchronize()
    assert resumed.epochs == full.epochs == 2 and resumed.iterations == full.iterations == 4
    for na, nb in ((full.generator, resumed.generator), (full.discriminator, resumed.discriminator)):
        for t in ("data", "m", "v", "iterations"):
            assert torch.equal(getattr(na.arena, t), getattr(nb.arena, t)), t
        for k, v in na.bn.export().items():
            assert np.array_equal(v, nb.bn.export()[k]), k
    assert (tmp_path / "b" / "models" / "pix2pix.npz").exists()
    assert (tmp_path / "a" / "logs" / "train_1" / "events.jsonl").exists()


@gpu
@pytest.mark.parametrize("C", [1, 3, 4])
def test_stage_pair_and_strided_copy_are_exact_copies(C):
    """dg_stage_pair (the step's input staging: concatenate([inp, tar]) at pix2pix.py:200, D(fake)'s
    x half, the identity pass's [x; y] batch) and dg_strided_copy's few-channel path move bits."""
    from dgan import ops
    g = torch.Generator().manual_seed(C)
    x = torch.randn(3, 17, 19, C, generator=g).cuda()
    y = torch.randn(3, 17, 19, C, generator=g).cuda()
    cat = torch.full((3, 17, 19, 2 * C + 1), 7.0, device="cuda")
    catx = torch.full((3, 17, 19, 2 * C), 7.0, device="cuda")
    gin = torch.full((6, 17, 19, C), 7.0, device="cuda")
    ops.stage_pair(x, y, cat[..., :2 * C], catx[..., :C], gin[:3], gin[3:])
    ops.strided_copy(y, catx[..., C:])
    torch.cuda.synchronize()
    assert torch.equal(cat[..., :C], x) and torch.equal(cat[..., C:2 * C], y)
    assert torch.equal(cat[..., 2 * C], torch.full_like(cat[..., 2 * C], 7.0))   # untouched column
    assert torch.equal(catx, torch.cat([x, y], -1))
    assert torch.equal(gin, torch.cat([x, y], 0))
    cat2 = torch.zeros(3, 17, 19, 2 * C, device="cuda")
    ops.stage_pair(x, y, cat2)   # optional outputs absent
    torch.cuda.synchronize()
    assert torch.equal(cat2, torch.cat([x, y], -1))
