"""The data-parallel step on RCCL itself (torch.distributed backend "nccl" on
ROCm), on the box's one MI355X: a world-size-1 process group in a fresh child
process, the same `dgan.dist.GradSync` hooks BASELINE configs[3] / [4] run on
8 GPUs (train_pix2pix.py:64-69 all-reduced; train_fsrgan.py's step likewise).

What runs: pix2pix full width at 256x256 bs2 with the VGG19 content term, and
FastSRGAN at its BASELINE image size 128 -> 512 (bs2), each with small buckets
so several all-reduces are issued while the generator's backward is still
being enqueued; one eager step, then the step captured ONCE in a HIP graph
(the RCCL collectives and the bucket hooks inside it) and replayed twice.

What is checked: at world size 1 the all-reduce is the identity and Adam's
1/world scale is 1, so every G / D parameter, gradient, Adam slot and BN
moving statistic after the three steps is bit-identical to the same three
steps without the process group."""
import contextlib
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

gpu = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Args:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _model(kind):
    if kind == "pix2pix":
        from pix2pix import Pix2Pix
        return Pix2Pix(Args(crop_size=256, retrain=0, width=1, seed=21, dropout_seed=0, identity_loss=1,
                            content_loss=1))
    from fsrgan import FastSRGAN
    return FastSRGAN(Args(crop_size=512, scale=4, fp16=0, lr=1e-3, seed=21, retrain=0, content_loss=1,
                          vgg_width=8))


def _data(kind):
    from dataloader import synthetic_pair
    if kind == "pix2pix":
        return synthetic_pair(2, 256, seed=77)
    x, y = synthetic_pair(2, 512, seed=77)
    return np.ascontiguousarray(x[:, ::4, ::4]), y


def _run(kind, dp, bucket_bytes):
    m = _model(kind)
    sync = None
    if dp:
        from dgan.dist import setup_data_parallel
        sync = setup_data_parallel(m, bucket_bytes=bucket_bytes)
    x, y = (torch.from_numpy(a).cuda() for a in _data(kind))
    tr = m.trainer(x.shape) if kind == "pix2pix" else m.trainer(x.shape, y.shape)
    assert tr.grad_sync is sync
    cur = torch.cuda.current_stream()
    s = torch.cuda.Stream()
    s.wait_stream(cur)
    with torch.cuda.stream(s):
        tr.step(x, y)                      # eager step (builds every lazily sized buffer)
    cur.wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    # (no settling delay: the captured all-reduces run on the capture-only group, dist.capture_group,
    # and the capture is thread-local, dist.CAPTURE_MODE)
    from dgan.dist import CAPTURE_MODE
    with (sync.capturing() if dp else contextlib.nullcontext()):
        with torch.cuda.graph(g, capture_error_mode=CAPTURE_MODE):
            tr.step(x, y)                  # captured once: RCCL all-reduces + bucket hooks inside
    torch.cuda.synchronize()
    counts = (sync.last_mid_backward, sync.last_total) if sync else None
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    out = {}
    for tag, net in (("G", m.generator), ("D", m.discriminator)):
        A = net.arena
        for slot in ("data", "grad", "m", "v"):
            out[f"{tag}.{slot}"] = getattr(A, slot).clone()
        out[f"{tag}.iterations"] = A.iterations.clone()
        for i, t in enumerate(net.non_trainable_variables):
            out[f"{tag}.bn{i}"] = t.clone()
    out["loss"] = tr.loss.clone()
    del g
    return out, counts


def _worker(port, q):
    for p in (os.path.join(REPO, "denoise-gan_amd"), REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    res = {"backend": dist.get_backend()}
    try:
        for kind, bucket in (("pix2pix", 8 << 20), ("fsrgan", 64 << 10)):
            ref, _ = _run(kind, dp=False, bucket_bytes=bucket)
            got, counts = _run(kind, dp=True, bucket_bytes=bucket)
            mism = [k for k in ref if not torch.equal(ref[k], got[k])]
            res[kind] = {"mismatch": mism, "counts": counts, "n": len(ref),
                         "loss": [float(v) for v in got["loss"].cpu()]}
            del ref, got
            torch.cuda.empty_cache()
        q.put(res)
    except Exception as e:  # report to the parent, then fail this process
        q.put({"error": repr(e)})
        raise
    finally:
        dist.destroy_process_group()


@gpu
def test_rccl_world1_graph_captured_step_bit_identical():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=300)
    p.join(timeout=60)
    assert "error" not in res, res
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    for kind in ("pix2pix", "fsrgan"):
        r = res[kind]
        assert r["mismatch"] == [], (kind, r["mismatch"])
        mid, total = r["counts"]
        # D's arena plus several G buckets go out before the backward's last layer
        assert mid >= 3 and total > mid, (kind, r["counts"])
        assert all(np.isfinite(r["loss"])), (kind, r["loss"])


@gpu
def test_bench_dist_world1_uses_rccl():
    """`bench.py --dist` at world size 1: the process group + RCCL path with the
    step graph-captured; one JSON line, dp1.  (Not --profile-only: that mode skips the
    graph-vs-eager check, whose snapshot kernels would land in a profile.)"""
    env = dict(os.environ, MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--dist", "--steps", "3", "--warmup", "2",
                        "--batch", "4", "--no-cpu-baseline", "--no-pmc-leg", "--no-core", "--no-twin"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["config"]["parallelism"] == "dp1" and out["config"]["process_group"] == "nccl", out["config"]
    assert out["config"]["hip_graph"] is True
    # (the data-parallel path replays the captured graph at every N since round 6; its replay equals
    # the eager step with its RCCL all-reduces, bit for bit)
    assert out["graph_equals_eager"]["equal"] is True, out["graph_equals_eager"]
    assert out["value"] > 0


def test_bench_refuses_gpus_without_launcher():
    """--gpus N > 1 without torch.distributed.run (no WORLD_SIZE) must fail, not
    measure one GPU and label it N (CPU: exits before touching a device)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert "torch.distributed.run" in r.stderr
