"""BASELINE.json configurations at full size, checked through size-independent
properties (the fp64 oracle is checked at reduced sizes in test_sr_gpu.py /
test_step_gpu.py):

  * every loss finite, generator output in (-1, 1);
  * bitwise determinism: two fresh models with the same seed produce
    identical losses, generator outputs and gradient arenas (all reductions
    in the library are fixed-order);
  * one Adam step at a small learning rate lowers the generator's own
    objective (gen_total - adv: content + mae, whose value depends on G only)
    on the same batch -- the step is a descent step.

Configs (BASELINE.json): SRGAN 4x 24->96 bs32 with 16 residual blocks;
FastSRGAN 128->512 bs8; Autoencoder 64x64 bs4 (grayscale replicated to 3
channels); pix2pix 256x256 bs16 is the bench workload (bench.py).
"""
import numpy as np
import pytest
import torch

gpu = pytest.mark.gpu


class Args:
    def __init__(self, **kw):
        self.fp16 = 0
        self.lr = 1e-3
        self.retrain = 0
        self.seed = 5
        self.__dict__.update(kw)


def _batch(N, H, scale, gray=False, seed=0):
    from dataloader import synthetic_pair
    x, y = synthetic_pair(N, H, seed=seed)
    if gray:  # BASELINE config a: grayscale, replicated to the model's 3 channels
        y = np.repeat(y.mean(axis=-1, keepdims=True), 3, axis=-1).astype(np.float32)
        x = np.repeat(x.mean(axis=-1, keepdims=True), 3, axis=-1).astype(np.float32)
    if scale > 1:
        x = np.ascontiguousarray(x[:, ::scale, ::scale, :])
    return torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()


def _one_step(cls, H, scale, N, gray=False, lr=1e-3):
    m = cls(Args(crop_size=H, scale=scale, lr=lr))
    x, y = _batch(N, H, scale, gray)
    tr = m.trainer(x.shape, y.shape)
    loss = tr.step(x, y, apply=False).clone()
    torch.cuda.synchronize()
    return m, tr, x, y, loss


def _check(cls, H, scale, N, gray=False):
    m1, tr1, x, y, l1 = _one_step(cls, H, scale, N, gray)
    assert torch.isfinite(l1).all(), l1
    gen = tr1.gen_output
    assert float(gen.abs().max()) < 1.0
    g1 = m1.generator.arena.grad.clone()
    d1 = m1.discriminator.arena.grad.clone()
    gen1 = gen.clone()
    del tr1
    m2, tr2, _, _, l2 = _one_step(cls, H, scale, N, gray)
    assert torch.equal(l1, l2)
    assert torch.equal(gen1, tr2.gen_output)
    assert torch.equal(g1, m2.generator.arena.grad)
    assert torch.equal(d1, m2.discriminator.arena.grad)
    del tr2
    # descent on a fixed batch
    m3, tr3, _, _, l3 = _one_step(cls, H, scale, N, gray, lr=1e-5)
    before = float(l3[0] - l3[1])
    tr3.step(x, y)             # with the Adam update
    after = tr3.step(x, y, apply=False)
    torch.cuda.synchronize()
    assert float(after[0] - after[1]) < before, (before, float(after[0] - after[1]))


@gpu
def test_srgan_full_config_bs32_24_to_96():
    from srgan import SRGAN
    _check(SRGAN, 96, 4, 32)


@gpu
def test_fsrgan_full_config_bs8_128_to_512():
    from fsrgan import FastSRGAN
    _check(FastSRGAN, 512, 4, 8)


@gpu
def test_autoencoder_config_64_gray_bs4():
    from autoencoder import Autoencoder
    _check(Autoencoder, 64, 1, 4, gray=True)


@gpu
def test_pix2pix_full_config_bs16_deterministic():
    from pix2pix import Pix2Pix

    def run():
        m = Pix2Pix(Args(crop_size=256, width=1, seed=3, dropout_seed=1))
        x, y = _batch(16, 256, 1, seed=4)
        tr = m.trainer(x.shape)
        loss = tr.step(x, y, apply=False).clone()
        torch.cuda.synchronize()
        return m, loss

    m1, l1 = run()
    assert torch.isfinite(l1).all() and float(l1[4]) > 0.0   # content term on (VGG19)
    g1 = m1.generator.arena.grad.clone()
    del m1
    m2, l2 = run()
    assert torch.equal(l1, l2)
    assert torch.equal(g1, m2.generator.arena.grad)
