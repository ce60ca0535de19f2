"""The data-parallel training step end to end on the HIP path: two ranks on
the box's one GPU, gloo as the transport (RCCL needs one GPU per rank; the
collective calls, the bucket hooks and the 1/world Adam scale are the same
code the 8-GPU RCCL run uses, dgan/dist.py).

Each rank trains on its own batch; after one step both ranks must hold
identical parameters, equal to Keras-Adam applied to the mean of the two
ranks' single-process gradients (BN statistics are per replica)."""
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


def _worker(rank, world, port, q):
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
        from pix2pix import Pix2Pix
        from dgan.dist import setup_data_parallel
        m = Pix2Pix(Args())
        setup_data_parallel(m, bucket_bytes=1 << 20)
        x, y = _batch(rank)
        loss = m.trainer(x.shape).step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda())
        torch.cuda.synchronize()
        q.put((rank, m.generator.arena.data.cpu().numpy(), m.discriminator.arena.data.cpu().numpy(),
               loss.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@gpu
def test_data_parallel_step_two_ranks_matches_mean_gradient():
    import torch.multiprocessing as mp
    from pix2pix import Pix2Pix
    from dgan import ops
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # replicas agree bit-for-bit (all-reduced gradients, identical Adam)
    assert np.array_equal(res[0][1], res[1][1])
    assert np.array_equal(res[0][2], res[1][2])
    # expected: Adam on the mean of the single-process gradients of the two batches
    grads_g, grads_d = [], []
    for r in range(world):
        m = Pix2Pix(Args())
        x, y = _batch(r)
        m.trainer(x.shape).step(torch.from_numpy(x).cuda(), torch.from_numpy(y).cuda(), apply=False)
        torch.cuda.synchronize()
        grads_g.append(m.generator.arena.grad.clone())
        grads_d.append(m.discriminator.arena.grad.clone())
    m = Pix2Pix(Args())
    for A, gs in ((m.generator.arena, grads_g), (m.discriminator.arena, grads_d)):
        A.grad.copy_(gs[0] + gs[1])
        ops.adam(A.data, A.grad, A.m, A.v, 2e-4, 0.5, 0.999, 1e-7, A.iterations, grad_scale=0.5)
    torch.cuda.synchronize()
    for got, want in ((res[0][1], m.generator.arena.data.cpu().numpy()),
                      (res[0][2], m.discriminator.arena.data.cpu().numpy())):
        d = np.abs(got - want)
        # fp32 sum order of the all-reduce vs the local sum: ulp-level gradient
        # differences, amplified at most to one Adam step (lr) where g ~ 0
        assert d.max() <= 2e-4 + 1e-7, d.max()
        assert np.median(d) < 1e-7
