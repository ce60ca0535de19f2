"""The fused pix2pix training step (train_pix2pix.py:33-71) on libdgan.

One call = the reference's traced `train_step`:
  G(x) [slot 0], G(y) [slot 1, identity loss pix2pix.py:90], D([x,y]),
  D([x,G(x)]), the 8 loss values, the D-loss backward through both D
  passes, the G-loss backward through D(fake) into G (both G passes), the
  data-parallel gradient all-reduce, then Keras-Adam on G and on D.
Both "tapes" see the same pre-update weights, as in the reference.

Everything is enqueued on the current stream with pre-sized buffers and a
pre-sized workspace, so a whole step can be captured in a HIP graph.
"""
import os

import torch

from . import ops
from .nets import DiscriminatorPlan, GeneratorPlan, DROP_RATE

# D's parameter backward (both halves) on a second stream beside the G path (D(fake)'s input
# gradient, the VGG19 backward, G's backward): the two are independent until Adam, and the D
# pass's small grids, BN passes and tails fill the G path's idle CU slots.  DG_NO_OVERLAP: one
# stream (same-box A/B)
OVERLAP = not os.environ.get("DG_NO_OVERLAP")
# ... and D's forward beside the VGG19 content forward (DG_NO_OVERLAP_DF: in sequence)
OVERLAP_DF = not os.environ.get("DG_NO_OVERLAP_DF")
# ... and D(fake)'s input gradient (the G path through D) on a third stream beside the VGG19
# backward, into its own buffer added to dL/dG(x) at the join (DG_NO_OVERLAP_DH: in sequence)
OVERLAP_DH = not os.environ.get("DG_NO_OVERLAP_DH")
# ... and (one process, no all-reduce) G's Adam over the arena prefix of 'last' and the up blocks --
# the backward-completion layout puts them first, final once up1's backward is enqueued -- on a
# stream beside the down blocks' backward; the down blocks' suffix after it (DG_NO_EARLY_ADAM: one
# Adam launch per network after the backward)
EARLY_ADAM = not os.environ.get("DG_NO_EARLY_ADAM")
# ... and the target's VGG19 forward (its own N-image plan) on a stream beside the generator's
# forward from the start of the step (DG_NO_OVERLAP_VT: one 2N VGG19 forward after G)
OVERLAP_VT = not os.environ.get("DG_NO_OVERLAP_VT")
# D's parameter backward forked at the start of G's backward instead of after the losses
DBWD_LATE = bool(os.environ.get("DG_DBWD_LATE"))
# the step's input staging in one launch (dg_stage_pair) instead of a concat and three copies;
# DG_STAGE_SPLIT=1: the four launches (same-box A/B)
STAGE_SPLIT = bool(os.environ.get("DG_STAGE_SPLIT"))

LOSS_NAMES = ("gen_total_loss", "gen_gan_loss", "gen_l1_loss", "gen_l2_loss", "content_loss", "disc_loss",
              "var_loss", "identity_loss")


def state_tensors(tr):
    """name -> device tensor of everything a training step carries to the next one or returns:
    both networks' parameter, gradient and Adam arenas and iteration counters, the BN moving
    statistics, the loss vector and (mixed_float16) the loss-scale states.  Works on a
    Pix2PixTrainer and on an SRTrainer (dgan.sr_trainer): for comparing two ways of running the
    same step (graph replay vs eager launches, one stream vs several) from one starting state."""
    nets = (("G", tr.gA, tr.G.bn), ("D", tr.dA, tr.D.bn)) if hasattr(tr, "gA") else \
        (("G", tr.G.arena, tr.G.bn), ("D", tr.D.arena, tr.D.bn))
    out = {}
    for tag, A, bn in nets:
        for k in ("data", "grad", "m", "v", "iterations"):
            out[f"{tag}.{k}"] = getattr(A, k)
        for k in bn.mean:
            out[f"{tag}.bn.{k}.mean"] = bn.mean[k]
            out[f"{tag}.bn.{k}.var"] = bn.var[k]
    out["loss"] = tr.loss
    for k in ("ls_g", "ls_d"):
        if getattr(tr, k, None) is not None:
            out[k] = getattr(tr, k)
    return out


def snapshot(tr):
    """Copies of state_tensors(tr) (enqueued on the current stream)."""
    return {k: t.clone() for k, t in state_tensors(tr).items()}


def restore(tr, snap):
    """Write a snapshot back into the trainer's own tensors (addresses unchanged: a captured
    graph of the step stays valid)."""
    for k, t in state_tensors(tr).items():
        t.copy_(snap[k])


def state_diff(a, b):
    """Names whose tensors differ in any bit between two snapshots."""
    return [k for k in a if not torch.equal(a[k], b[k])]


class AdamConfig:
    def __init__(self, lr=2e-4, beta_1=0.5, beta_2=0.999, epsilon=1e-7):
        self.lr, self.beta_1, self.beta_2, self.epsilon = lr, beta_1, beta_2, epsilon

    def current_lr(self):
        return float(self.lr)


class Pix2PixTrainer:
    """One fused pix2pix step for x, y [N,H,W,3].

    The two generator calls (G(x) and the identity pass G(y)) run as ONE
    U-Net pass over 2N images, and the two discriminator calls (real, fake)
    as one PatchGAN pass over 2N images; BatchNorm statistics, moving
    averages and dropout stay per call (GeneratorPlan / DiscriminatorPlan
    `halves`).  Backward: one G pass over both halves (their gradients sum,
    as the reference's single gen_tape does over the two calls), one D pass
    over both halves for the disc gradients, and the G-path gradient through
    D(fake) on the fake half only."""

    def __init__(self, g_arena, g_bn, d_arena, d_bn, N, H, W, device, width=1, identity=True,
                 loss_weights=ops.LOSS_WEIGHTS_REF, drop_rate=DROP_RATE, drop_seed=0, g_opt=None, d_opt=None,
                 grad_sync=None, vgg=None):
        self.gA, self.dA = g_arena, d_arena
        self.N, self.H, self.W = N, H, W
        self.identity = identity
        self.weights = tuple(loss_weights)
        self.drop_rate, self.drop_seed = drop_rate, drop_seed
        self.g_opt = g_opt or AdamConfig()
        self.d_opt = d_opt or AdamConfig()
        self.grad_sync = grad_sync
        gh = 2 if identity else 1
        self.G = GeneratorPlan(N, H, W, width, g_arena, g_bn, device, halves=gh, train=True)
        self.D = DiscriminatorPlan(N, H, W, width, d_arena, d_bn, device, halves=2, train=True)
        lshape = (N,) + tuple(self.D.out_shape[1:])
        e = lambda shape: torch.empty(shape, dtype=torch.float32, device=device)
        self.gin = e((gh * N, H, W, 3)) if identity else None   # [x; y]
        self.gout = e((gh * N, H, W, 3))                        # [G(x); G(y)]
        self.dgout = e((gh * N, H, W, 3))                       # [dL/dG(x); dL/dG(y)]
        self.dlog = e(self.D.out_shape)                         # [dzr_d; dzf_d]
        self.dzf_g = e(lshape)
        self.dinp = e((N, H, W, 6))                             # dL/d D([x, G(x)]) of the G path
        self.loss = torch.zeros(8, dtype=torch.float32, device=device)
        # VGG19 content loss (pix2pix.py:45-51, :87): frozen feature extractor on G(x) and y
        self.content = None
        # (the split VGG19 plans also when the step runs on one stream -- profiling, DG_NO_OVERLAP --
        # so the one-stream step runs the overlapped step's kernels: the two are bit-identical,
        # tests/test_overlap_gpu.py)
        vsplit = OVERLAP_VT
        if vgg is not None and self.weights[5] != 0.0:
            from .sr_trainer import ContentLoss
            self.content = ContentLoss(vgg, N, H, W, device, split=vsplit)
        ws_bytes = max(self.G.ws_bytes, self.D.ws_bytes,
                       ops.p2p_loss_workspace_bytes(N, H, W, 3, lshape[0] * lshape[1] * lshape[2]),
                       self.content.ws_bytes if self.content else 0)
        self.ws = ops.Workspace(device)
        self.ws.get(ws_bytes)
        # the side stream of the overlapped D parameter backward, with its own workspace
        self.side = None
        if OVERLAP and getattr(self.D, "dz_h", None) is not None:
            self.side = torch.cuda.Stream(device=device)
            self.ws_side = ops.Workspace(device)
            self.ws_side.get(self.D.ws_bytes)
        # G arena prefix final after the up blocks' backward (layout = backward completion order)
        downs = {n for n, *_ in self.G.downs}
        self.g_split = min(g_arena.offsets[n] for n in g_arena.layout if n.split("/")[0] in downs)
        assert all(g_arena.end_offset(n) <= self.g_split for n in g_arena.layout if n.split("/")[0] not in downs)
        self.g_last_up = self.G.ups[0][0]   # (G.backward's last up block)
        self.side4 = None
        if self.side is not None and self.content is not None and self.content.split:
            self.side4 = torch.cuda.Stream(device=device)
            self.ws_vgg = ops.Workspace(device)
            self.ws_vgg.get(self.content.tws_bytes)
        self.side3 = None
        if self.side is not None and EARLY_ADAM:
            self.side3 = torch.cuda.Stream(device=device)
        self.side2 = None
        # D(fake)'s input gradient into its own buffer, added to dL/dG(x) after the VGG19 backward
        # -- on side2 beside that backward, or in sequence on one stream (the same additions in the
        # same order either way)
        self.dgen_d = None
        if OVERLAP_DH and self.content is not None and self.D.desc_g3 is not None:
            self.dgen_d = e((N, H, W, 3))
            if self.side is not None:
                self.side2 = torch.cuda.Stream(device=device)
                self.ws_side2 = ops.Workspace(device)
                self.ws_side2.get(self.D.ws_bytes)

    @property
    def gen_output(self):
        """G(x) of the last step."""
        return self.gout[:self.N]

    def step(self, x, y, apply=True):
        """x, y: device NHWC [N,H,W,3] fp32 in [-1, 1].  Returns the 8 losses (device, no sync)."""
        x = x if x.is_contiguous() else x.contiguous()
        y = y if y.is_contiguous() else y.contiguous()
        ws = self.ws
        G, D = self.G, self.D
        N = self.N
        inp = D.inp
        real_in, fake_in = inp[:N], inp[N:]
        step_dev = self.gA.iterations
        main = torch.cuda.current_stream()
        # the target's VGG19 features (pix2pix.py:45-51: vgg(pre(target))) need nothing of G:
        # beside G's forward on side4 once the shared weight planes are settled
        tfork = False
        if self.content is not None and self.content.split:
            tfork = self.side4 is not None and not ops.profiling() and self.content.settled()
            if tfork:
                self.side4.wait_stream(main)
                with torch.cuda.stream(self.side4):
                    self.content.forward_target(y, ws=self.ws_vgg)
            else:
                self.content.forward_target(y, ws=ws)
        # ---- forward (pix2pix.py:44-48 and the identity pass :90) -----------
        # concatenate([inp, tar]) (pix2pix.py:200), D(fake)'s x half, and the identity pass's
        # [x; y] G batch (pix2pix.py:44,90): one staging launch
        if STAGE_SPLIT:
            ops.channel_concat(x, y, real_in)
            ops.strided_copy(x, fake_in[..., :3])
            if self.identity:
                ops.strided_copy(x, self.gin[:N])
                ops.strided_copy(y, self.gin[N:])
            gin = self.gin if self.identity else x
        elif self.identity:
            ops.stage_pair(x, y, real_in, fake_in[..., :3], self.gin[:N], self.gin[N:])
            gin = self.gin
        else:
            ops.stage_pair(x, y, real_in, fake_in[..., :3])
            gin = x
        G.forward(gin, self.gout, ws=ws, drop_rate=self.drop_rate, drop_seed=self.drop_seed, step_dev=step_dev)
        gen = self.gout[:N]
        ident = self.gout[N:] if self.identity else None
        ops.strided_copy(gen, fake_in[..., 3:])
        side = self.side if not ops.profiling() else None
        content = None
        tsync = (lambda: main.wait_stream(self.side4)) if tfork else None
        if side is not None and OVERLAP_DF and self.content is not None:
            # D's forward on the side stream beside the VGG19 forward (both read G(x) only; the
            # losses join them)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                logits = D.forward(ws=self.ws_side)
            content = self.content.forward(gen, y, grad_weight=self.weights[5], ws=ws, tsync=tsync)
            main.wait_stream(side)
        else:
            logits = D.forward(ws=ws)
            if self.content is not None:
                # content_loss(target, gen) = MSE(vgg(pre(y))/12.75, vgg(pre(G(x)))/12.75) (pix2pix.py:45-51)
                content = self.content.forward(gen, y, grad_weight=self.weights[5], ws=ws, tsync=tsync)
        zr, zf = logits[:N], logits[N:]
        # ---- losses + their gradients (pix2pix.py:74-103) ----------------
        dgen = self.dgout[:N]
        ops.p2p_loss(gen, y, zr, zf, self.loss, ident=ident, weights=self.weights, content=content,
                     dgen=dgen, dident=self.dgout[N:] if self.identity else None, dlogit_real_d=self.dlog[:N],
                     dlogit_fake_d=self.dlog[N:], dlogit_fake_g=self.dzf_g, ws=ws)
        sync = self.grad_sync
        # ---- disc_tape.gradient (train_pix2pix.py:65): both D calls in one pass
        def d_param_backward():
            # (on the side stream; its all-reduce is issued from there)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                D.backward(self.dlog, param_grads=True, beta=0.0, ws=self.ws_side)
                if sync:
                    sync.start("D")
        dlate = side is not None and DBWD_LATE
        if side is not None and not dlate:
            d_param_backward()   # (forked after the losses)
        elif side is None:
            D.backward(self.dlog, param_grads=True, beta=0.0, ws=ws)
            if sync:
                sync.start("D")
        # ---- gen_tape.gradient (train_pix2pix.py:64): through D(fake) into G(x)
        side2 = self.side2 if side is not None else None
        if side2 is not None:
            # D(fake)'s input gradient beside the VGG19 backward (which accumulates into dgen
            # meanwhile): into dgen_d, added at the join
            side2.wait_stream(main)
            with torch.cuda.stream(side2):
                D.backward(self.dzf_g, half=1, param_grads=False, input_grad=self.dgen_d, input_beta=0.0,
                           ws=self.ws_side2, input_from=3)
            self.content.backward(dgen, beta=1.0, ws=ws)
            main.wait_stream(side2)
            ops.accumulate(self.dgen_d, dgen, 1.0)
        elif self.dgen_d is not None:   # (the same on one stream)
            D.backward(self.dzf_g, half=1, param_grads=False, input_grad=self.dgen_d, input_beta=0.0, ws=ws,
                       input_from=3)
            self.content.backward(dgen, beta=1.0, ws=ws)
            ops.accumulate(self.dgen_d, dgen, 1.0)
        else:
            if D.desc_g3 is not None:   # dL/dG(x) += channels 3..5 of dL/d D([x, G(x)])
                D.backward(self.dzf_g, half=1, param_grads=False, input_grad=dgen, input_beta=1.0, ws=ws,
                           input_from=3)
            else:
                D.backward(self.dzf_g, half=1, param_grads=False, input_grad=self.dinp, input_beta=0.0, ws=ws)
                ops.accumulate(self.dinp[..., 3:], dgen, 1.0)
            if self.content is not None:
                self.content.backward(dgen, beta=1.0, ws=ws)
        # both generator calls (G(x), G(y)) in one backward: their gradients sum
        early = apply and sync is None and self.side3 is not None and side is not None
        hook = sync.ready_G if sync else None
        if early:
            side3, gA, go = self.side3, self.gA, self.g_opt

            def hook(name):
                if name != self.g_last_up:
                    return
                # the up blocks' gradients are enqueued: their Adam beside the down blocks' backward
                k = self.g_split
                side3.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side3):
                    ops.adam(gA.data[:k], gA.grad[:k], gA.m[:k], gA.v[:k], go.current_lr(), go.beta_1, go.beta_2,
                             go.epsilon, gA.iterations)
        if dlate:
            d_param_backward()   # (forked at G's backward: its small layers leave CUs to fill)
        G.backward(self.dgout, beta=0.0, ws=ws, drop_rate=self.drop_rate, on_grads_ready=hook)
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)   # (join: D's gradients before Adam)
        if sync:
            sync.finish()
        # ---- apply_gradients (train_pix2pix.py:68-69) ----------------------
        if self.content is not None and self.content.split:
            self.content.mark_settled()
        if apply:
            scale = sync.grad_scale if sync else 1.0
            # the optimizers' hyper-parameters are read at every step (a changed or callable
            # learning_rate takes effect; a captured HIP graph keeps the values of its capture)
            for A, o in ((self.gA, self.g_opt), (self.dA, self.d_opt)):
                if early and A is self.gA:   # (the prefix ran on side3; the suffix here, then the join)
                    k = self.g_split
                    ops.adam(A.data[k:], A.grad[k:], A.m[k:], A.v[k:], o.current_lr(), o.beta_1, o.beta_2,
                             o.epsilon, A.iterations)
                    torch.cuda.current_stream().wait_stream(self.side3)
                else:
                    ops.adam(A.data, A.grad, A.m, A.v, o.current_lr(), o.beta_1, o.beta_2, o.epsilon,
                             A.iterations, grad_scale=scale)
                ops.counter_add(A.iterations, 1)
        return self.loss
