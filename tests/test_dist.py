"""Data-parallel gradient exchange (dgan/dist.py) on CPU with gloo, world_size 2.

Each rank fills its G and D gradient arenas with rank-specific values, runs
the same hook sequence the trainer runs (D all-reduce after D's backward,
G buckets issued as layers complete in backward order, finish before Adam)
and checks the summed arenas, the 1/world scale, and that bucket boundaries
follow the arena's backward-completion layout."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, width, bucket_bytes, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dgan.nets import Arena, d_layout_order, d_variables, g_layout_order, g_layer_specs, g_variables
        from dgan.dist import GradSync
        gA = Arena(g_variables(width), torch.device("cpu"), g_layout_order(width))
        dA = Arena(d_variables(width), torch.device("cpu"), d_layout_order(width))
        g = torch.arange(gA.numel, dtype=torch.float32) * 1e-3 + rank
        d = torch.arange(dA.numel, dtype=torch.float32) * 1e-3 - rank
        gA.grad.copy_(g)
        dA.grad.copy_(d)
        sync = GradSync(gA, dA, bucket_bytes=bucket_bytes)
        sync.start("D")
        downs, ups, last = g_layer_specs(width)
        issued = []
        for layer in ["last"] + [u[0] for u in reversed(ups)] + [dn[0] for dn in reversed(downs)]:
            before = sync.issued
            sync.ready_G(layer)
            if sync.issued != before:
                issued.append((before, sync.issued))
        sync.finish()
        q.put((rank, gA.grad.numpy().copy(), dA.grad.numpy().copy(), sync.grad_scale, issued, gA.numel))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_kb", [256, 65536])
def test_gradsync_two_ranks(bucket_kb):
    width = 8
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, width, bucket_kb << 10, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    n = res[0][5]
    g_expect = (np.arange(n, dtype=np.float32) * 1e-3) * 2 + 1.0
    for rank, g, d, scale, issued, _ in res:
        assert scale == 0.5
        assert np.allclose(g, g_expect, rtol=1e-6)
        d_expect = (np.arange(d.size, dtype=np.float32) * 1e-3) * 2 - 1.0
        assert np.allclose(d, d_expect, rtol=1e-6, atol=1e-6)
        # buckets are contiguous, ascending, and start at 0
        pos = 0
        for a, b in issued:
            assert a == pos and b > a
            pos = b
    # the small bucket size must have produced several in-flight buckets
    if bucket_kb == 256:
        assert len(res[0][4]) >= 3


def _sr_worker(rank, world, port, kind, bucket_bytes, q):
    """GradSync over a dgan.graph network arena, driven by the layer names the
    graph executor's backward reports (GraphPlan.backward -> on_grads_ready)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dgan import zoo
        from dgan.dist import GradSync
        from dgan.nets import Arena
        g = zoo.srgan_generator(scale=4) if kind == "srgan" else zoo.fsrgan_generator()
        d = zoo.sr_discriminator(df=32)
        gA = Arena(g.var_list(), torch.device("cpu"), g.layout_order())
        dA = Arena(d.var_list(), torch.device("cpu"), d.layout_order())
        gA.grad.copy_(torch.arange(gA.numel, dtype=torch.float32) * 1e-3 + rank)
        dA.grad.copy_(torch.arange(dA.numel, dtype=torch.float32) * 1e-3 - rank)
        sync = GradSync(gA, dA, bucket_bytes=bucket_bytes)
        sync.start("D")
        issued = []
        for n in reversed(g.nodes[1:]):          # GraphPlan.backward's reporting order
            if n.kind in ("conv", "bn", "prelu", "dwconv"):
                before = sync.issued
                sync.ready_G(n.name)
                if sync.issued != before:
                    issued.append((before, sync.issued))
        sync.finish()
        q.put((rank, gA.grad.numpy().copy(), dA.grad.numpy().copy(), issued, gA.numel))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["srgan", "fsrgan"])
def test_gradsync_sr_graph_two_ranks(kind):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sr_worker, args=(r, world, port, kind, 64 << 10, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = res[0][4]
    for rank, g, d, issued, _ in res:
        assert np.allclose(g, np.arange(n, dtype=np.float32) * 2e-3 + 1.0, rtol=1e-6)
        assert np.allclose(d, np.arange(d.size, dtype=np.float32) * 2e-3 - 1.0, rtol=1e-6, atol=1e-6)
        pos = 0
        for a, b in issued:
            assert a == pos and b > a
            pos = b
        assert len(issued) >= 3   # buckets went out during the backward, not all at finish()
