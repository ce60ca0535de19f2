"""Data-parallel gradient exchange for the pix2pix step (one process per GPU).

The reference is single-GPU (train_pix2pix.py:15 pins CUDA_VISIBLE_DEVICES);
BASELINE.json's north star adds batch data parallelism: each rank runs the
full step on its own 16 images, then the fp32 gradient arenas are summed
with RCCL (torch.distributed backend "nccl" on ROCm) over xGMI and Adam
applies them scaled by 1/world (ops.adam grad_scale) on every rank, so the
replicas stay bit-identical without any parameter broadcast.

BatchNorm: the training step normalises with each replica's local batch
statistics (SyncBatchNorm is not used, as in tf.distribute's default), and
each replica updates its own moving averages from them.  Keras keeps those
moving variables ON_READ with MEAN aggregation, i.e. a read under
tf.distribute returns the cross-replica mean; `sync_bn_stats` performs that
read-time averaging (all-reduce mean of every moving mean / variance) and
the drivers call it before a checkpoint save or an inference read.

Overlap: D's gradients are final after the two D backwards and go out at
once (they travel while G's backward runs); G's arena is laid out in
backward-completion order (nets.g_layout_order), so a bucket is issued as
soon as the last layer inside it has its gradient enqueued.  The
collectives run on RCCL's own stream; `finish()` makes the compute stream
wait for them before Adam.
"""
import contextlib

import torch
import torch.distributed as dist


_CAPTURE_GROUPS = {}

# Capture mode of every HIP-graph capture of a step.  Under the default ("global") mode the HIP
# runtime refuses an event query from ANY thread while a capture is open
# (hipErrorStreamCaptureUnsupported), so a process group's watchdog that is still retiring the
# eager warm-up's all-reduces aborts the process (round 5: WorkNCCL::isCompleted on default_pg,
# once D's parameter backward moved to a side stream changed the warm-up's timing).  Thread-local
# mode restricts the check to the capturing thread; the watchdog's queries of events on the
# default group's stream (which never joins a capture, see capture_group) are then legal.
CAPTURE_MODE = "thread_local"


def capture_group(device=None):
    """The process group that carries only collectives issued inside HIP-graph capture.

    The watchdog thread of a process group queries the end event of every eager collective
    until it retires it; on ROCm that query fails with hipErrorCapturedEvent while the stream
    the event was recorded on is part of a capture, which aborts the process (round 4:
    WorkNCCL::isCompleted in test_bench_dist_world1_uses_rccl, after the eager warm-up's
    all-reduces were still listed when the captured step's all-reduces pulled RCCL's stream
    into the capture).  Collectives issued under capture are never listed (ProcessGroupNCCL
    enqueues a work for the watchdog only outside capture), so a group that runs nothing
    eagerly has nothing to query, whatever the timing: its RCCL stream is the only one that
    joins a capture, and the default group's eagerly recorded events stay on a stream that
    never does.  Created (collectively, by every rank) with its communicator connected eagerly
    (device_id), so no communicator is set up inside a capture."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    key = (dist.get_world_size(), str(device))
    if key not in _CAPTURE_GROUPS:
        _CAPTURE_GROUPS[key] = dist.new_group(backend=dist.get_backend(), device_id=device,
                                              group_desc="dgan_graph_capture")
    return _CAPTURE_GROUPS[key]


BUCKET_BYTES = 25 << 20   # ~25 MB buckets -> 9 G buckets + D for pix2pix


class GradSync:
    """Bucketed gradient all-reduce of one G and one D arena.  Works for any
    network whose backward reports finished layers by name (pix2pix plans,
    dgan.graph plans): a layer is the variable-name prefix before '/'."""

    def __init__(self, g_arena, d_arena, bucket_bytes=BUCKET_BYTES, group=None):
        self.g, self.d = g_arena, d_arena
        self.group = group
        self.world = dist.get_world_size(group)
        self.grad_scale = 1.0 / self.world
        self.bucket = max(1, bucket_bytes // 4)
        self.works = []
        self.issued = 0
        # all-reduces of the last step: issued before finish() (i.e. while the
        # backward was still being enqueued) and in total (D arena included)
        self.last_mid_backward = 0
        self.last_total = 0
        # arena end offset of every layer's last variable, in layout order
        self.layer_end = {}
        for name in g_arena.layout:
            layer = name.split("/")[0]
            self.layer_end[layer] = max(self.layer_end.get(layer, 0), g_arena.end_offset(name))

    def _reduce(self, t):
        self.works.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def start(self, which):
        if which == "D":
            self._reduce(self.d.grad)

    def ready_G(self, layer):
        end = self.layer_end[layer]
        if end - self.issued >= self.bucket:
            self._reduce(self.g.grad[self.issued:end])
            self.issued = end

    @contextlib.contextmanager
    def capturing(self, device=None):
        """Issue this sync's collectives on capture_group() for the duration (a HIP-graph capture
        of the step); the graph replays them there.  Every eager collective of the sync must have
        completed (finish()) -- they ran on the sync's own group."""
        if self.works:
            raise RuntimeError("GradSync.capturing: eager all-reduces still outstanding")
        group, self.group = self.group, (capture_group(device) if dist.get_backend(self.group) == "nccl"
                                         else self.group)
        try:
            yield self
        finally:
            self.group = group

    def finish(self):
        self.last_mid_backward = len(self.works)
        if self.issued < self.g.numel:
            self._reduce(self.g.grad[self.issued:])
        self.last_total = len(self.works)
        for w in self.works:
            w.wait()
        self.works.clear()
        self.issued = 0


def broadcast_parameters(model, src=0, group=None):
    """Make every rank start from rank src's weights (seeded init already agrees;
    this also covers restored checkpoints)."""
    for net in (model.generator, model.discriminator):
        dist.broadcast(net.arena.data, src, group=group)
        for t in net.non_trainable_variables:
            dist.broadcast(t, src, group=group)


def sync_bn_stats(model, group=None):
    """Cross-replica mean of every BN moving mean / variance (Keras ON_READ MEAN
    aggregation); identical on every rank afterwards."""
    world = dist.get_world_size(group)
    for net in (model.generator, model.discriminator):
        for t in net.non_trainable_variables:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            t.mul_(1.0 / world)


def setup_data_parallel(model, bucket_bytes=BUCKET_BYTES):
    """Attach the gradient exchange to a model container (Pix2Pix or an SR-family
    model) and broadcast rank 0's weights.  Trainers built before this call are
    dropped so every step built afterwards all-reduces."""
    model.grad_sync = GradSync(model.generator.arena, model.discriminator.arena, bucket_bytes)
    if hasattr(model, "_trainers"):
        model._trainers.clear()
    broadcast_parameters(model)
    return model.grad_sync
