#!/usr/bin/env python3
"""Gradient-bucket timeline of the pix2pix bs16 step (content on) on one GPU and
the predicted exposed all-reduce time at 8 GPUs (a model, not a measurement).

HIP events on the compute stream mark, inside the real step: the end of D's
backward (the D arena's all-reduce is issued there), the moment each 25 MB G
bucket becomes final (dgan.dist.GradSync's bucketing, same arena layout) and
the end of G's backward.  The modelled RCCL ring all-reduce of a bucket of b
bytes on p GPUs takes  lat + 2 (p-1)/p * b / busbw,  issued in order on one
comm stream as soon as it is ready.  Exposed communication = when the last
all-reduce ends minus when G's backward ends (what Adam would wait for).

    python scripts/diag/bucket_timeline.py > profiles/r3/bucket_timeline.txt
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO]

import torch  # noqa: E402

from dgan.dist import BUCKET_BYTES  # noqa: E402


class Timeline:
    """GradSync's interface (start / ready_G / finish), recording events instead of all-reducing."""

    def __init__(self, g_arena, d_arena, bucket_bytes=BUCKET_BYTES):
        self.g, self.d = g_arena, d_arena
        self.grad_scale = 1.0
        self.bucket = max(1, bucket_bytes // 4)
        self.layer_end = {}
        for name in g_arena.layout:
            layer = name.split("/")[0]
            self.layer_end[layer] = max(self.layer_end.get(layer, 0), g_arena.end_offset(name))
        self.reset()

    def reset(self):
        self.issued = 0
        self.marks = []   # (label, bytes, event)

    def _mark(self, label, nbytes):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self.marks.append((label, nbytes, e))

    def start(self, which):
        self._mark("D arena", self.d.grad.numel() * 4)

    def ready_G(self, layer):
        end = self.layer_end[layer]
        if end - self.issued >= self.bucket:
            self._mark(f"G bucket ..{layer}", (end - self.issued) * 4)
            self.issued = end

    def finish(self):
        if self.issued < self.g.numel:
            self._mark("G bucket (rest)", (self.g.numel - self.issued) * 4)
        self._mark("G backward end", 0)


def model_allreduce_us(nbytes, p, busbw, lat_us):
    return lat_us + 2.0 * (p - 1) / p * nbytes / busbw * 1e6


def main():
    from bench import Args, WORKLOADS, synthetic_batch
    from pix2pix import Pix2Pix
    m = Pix2Pix(Args(crop_size=256, retrain=0, width=1, seed=1234, dropout_seed=0, identity_loss=1, content_loss=1))
    tl = Timeline(m.generator.arena, m.discriminator.arena)
    m.grad_sync = tl
    x, y = (torch.from_numpy(t).cuda() for t in synthetic_batch(WORKLOADS["pix2pix"], 16, 1000))
    tr = m.trainer(x.shape)
    for _ in range(3):
        tl.reset()
        tr.step(x, y)
    torch.cuda.synchronize()
    reps = []
    for _ in range(5):
        tl.reset()
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record()
        tr.step(x, y)
        t1 = torch.cuda.Event(enable_timing=True)
        t1.record()
        torch.cuda.synchronize()
        reps.append(([(lab, nb, t0.elapsed_time(e)) for lab, nb, e in tl.marks], t0.elapsed_time(t1)))
    marks, step_ms = sorted(reps, key=lambda r: r[1])[len(reps) // 2]
    g_end = [t for lab, _, t in marks if lab == "G backward end"][0]
    print(f"pix2pix bs16 step (eager, content on): {step_ms:.3f} ms; G backward ends at {g_end:.3f} ms")
    print(f"{'bucket':28s} {'MB':>7s} {'ready (ms)':>11s} {'before G end (ms)':>18s}")
    buckets = [(lab, nb, t) for lab, nb, t in marks if nb > 0]
    for lab, nb, t in buckets:
        print(f"{lab:28s} {nb / 1e6:7.1f} {t:11.3f} {g_end - t:18.3f}")
    print()
    p = 8
    for busbw, lat in ((200e9, 30.0), (300e9, 25.0), (400e9, 20.0)):
        free, rows = 0.0, []
        for lab, nb, t in sorted(buckets, key=lambda b: b[2]):
            start = max(free, t * 1e3)
            free = start + model_allreduce_us(nb, p, busbw, lat)
            rows.append((lab, start / 1e3, free / 1e3))
        exposed = max(0.0, free / 1e3 - g_end)
        tot = sum(model_allreduce_us(nb, p, busbw, lat) for _, nb, _ in buckets) / 1e3
        pred = p * step_ms / (step_ms + exposed)
        print(f"model p={p}, RCCL busbw {busbw / 1e9:.0f} GB/s, {lat:.0f} us per collective: all-reduce total "
              f"{tot:.3f} ms, last one ends {free / 1e3:.3f} ms, exposed {exposed:.3f} ms -> predicted step "
              f"{step_ms + exposed:.3f} ms, {pred:.2f}x at {p} GPUs (weak scaling, no contention modelled)")


if __name__ == "__main__":
    main()
