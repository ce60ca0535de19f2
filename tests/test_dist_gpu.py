"""The data-parallel training step end to end on the HIP path: two ranks on
the box's one GPU, gloo as the transport (RCCL needs one GPU per rank; the
collective calls, the bucket hooks and the 1/world Adam scale are the same
code the 8-GPU RCCL run uses, dgan/dist.py).

pix2pix, SRGAN and FastSRGAN: the gradient exchange is checked bit-exactly on
the all-reduced arenas (apply=False), then a full step keeps the replicas
identical; BN moving statistics are averaged across replicas on demand
(dgan.dist.sync_bn_stats, Keras ON_READ MEAN)."""
import os
import socket

import numpy as np
import pytest
import torch

gpu = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Args:
    def __init__(self, **kw):
        self.crop_size = 256
        self.retrain = 0
        self.width = 8
        self.seed = 11
        self.dropout_seed = 0
        self.dropout_rate = 0.0
        self.content_loss = 0
        self.__dict__.update(kw)


def _batch(rank):
    from dataloader import synthetic_pair
    return synthetic_pair(2, 256, seed=300 + rank)


def _sr_args(kind):
    return dict(crop_size=32, scale=4, fp16=0, lr=1e-3, seed=11, vgg_width=8)


def _model(kind):
    if kind == "pix2pix":
        from pix2pix import Pix2Pix
        return Pix2Pix(Args())
    from fsrgan import FastSRGAN
    from srgan import SRGAN
    return (SRGAN if kind == "srgan" else FastSRGAN)(Args(**_sr_args(kind)))


def _data(kind, rank):
    x, y = _batch(rank)
    if kind != "pix2pix":
        from dataloader import synthetic_pair
        x, y = synthetic_pair(2, 32, seed=300 + rank)
        x = np.ascontiguousarray(x[:, ::4, ::4])
    return x, y


def _trainer(m, kind, x, y):
    return m.trainer(x.shape) if kind == "pix2pix" else m.trainer(x.shape, y.shape)


def _worker(rank, world, port, q, kind):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(repo, "denoise-gan_amd"), repo):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dgan.dist import setup_data_parallel, sync_bn_stats
        m = _model(kind)
        _trainer(m, kind, *_data(kind, rank))      # a trainer built before DP setup is dropped by it
        setup_data_parallel(m, bucket_bytes=1 << 20)
        x, y = _data(kind, rank)
        tr = _trainer(m, kind, x, y)
        assert tr.grad_sync is m.grad_sync
        xd, yd = torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda()
        tr.step(xd, yd, apply=False)               # gradients all-reduced (sum), no update
        torch.cuda.synchronize()
        grads = (m.generator.arena.grad.cpu().numpy(), m.discriminator.arena.grad.cpu().numpy())
        sync_bn_stats(m)
        bn = (m.generator.bn.export(), m.discriminator.bn.export())
        loss = tr.step(xd, yd)                     # a full step: replicas must stay identical
        torch.cuda.synchronize()
        q.put((rank, grads, bn, m.generator.arena.data.cpu().numpy(), m.discriminator.arena.data.cpu().numpy(),
               loss.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@gpu
@pytest.mark.parametrize("kind", ["pix2pix", "srgan", "fsrgan"])
def test_data_parallel_two_ranks(kind):
    """Two ranks on the one GPU, gloo transport.  The all-reduced gradient arenas are
    bit-equal to the sum of the two ranks' single-process gradients (a two-term fp32 sum
    is order-free), the BN moving statistics after sync_bn_stats equal the mean of the two
    single-process runs' statistics, and after a full step both replicas hold identical
    parameters (same all-reduced gradients, identical Adam with the 1/world scale)."""
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single_g, single_bn = [], []
    for r in range(world):
        m = _model(kind)
        x, y = _data(kind, r)
        _trainer(m, kind, x, y).step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), apply=False)
        torch.cuda.synchronize()
        single_g.append((m.generator.arena.grad.cpu().numpy(), m.discriminator.arena.grad.cpu().numpy()))
        single_bn.append((m.generator.bn.export(), m.discriminator.bn.export()))
    for rank in range(world):
        for k in range(2):
            assert np.array_equal(res[rank][1][k], single_g[0][k] + single_g[1][k]), (kind, rank, k)
            for name, v in res[rank][2][k].items():
                want = (single_bn[0][k][name].astype(np.float64) + single_bn[1][k][name]) / 2
                assert np.allclose(v, want, rtol=1e-6, atol=1e-7), (kind, name)
    assert np.array_equal(res[0][3], res[1][3]) and np.array_equal(res[0][4], res[1][4])
