"""Fused training steps of the SRGAN / FastSRGAN / Autoencoder families
(train_srgan.py:61-118, train_fsrgan.py:61-120, train_autoencoder.py:66-112)
on libdgan, and the VGG19 content loss shared with pix2pix.

One call = the reference's traced `train_step`:
  G(x); D(y) [slot 0], D(G(x)) [slot 1]; VGG19 on preprocess(G(x)) and
  preprocess(y) -> content MSE / 12.75; adv / mae / mse / tv / disc losses;
  the disc-loss backward through both D passes; the gen-loss backward
  through D(fake) and through VGG(G(x)) into G; Adam (ExponentialDecay,
  TTUR) on G and D.  Both gradients see the same pre-update weights, as in
  the reference's single persistent tape.

All launches go to the current stream with pre-sized buffers, so a step can
be captured in one HIP graph.
"""
import os

import torch

from . import ops
from .graph import GraphNetwork
from .zoo import vgg19_features

FEAT_SCALE = 1.0 / 12.75   # srgan.py:74-75


class ScheduleConfig:
    """keras.optimizers.schedules.ExponentialDecay + Adam hyper-parameters."""

    def __init__(self, lr, decay_steps=100000, decay_rate=0.1, staircase=True, beta_1=0.9, beta_2=0.999,
                 epsilon=1e-7):
        self.lr, self.decay_steps, self.decay_rate, self.staircase = lr, decay_steps, decay_rate, staircase
        self.beta_1, self.beta_2, self.epsilon = beta_1, beta_2, epsilon

    def __call__(self, step):
        e = step / self.decay_steps
        if self.staircase:
            e = float(int(e))
        return self.lr * self.decay_rate ** e


def apply_adam(arena, cfg, grad_scale=1.0, loss_scale=None):
    """loss_scale: the optimizer's device loss-scale state (fp16): the update is unscaled
    by it, or skipped with the iteration count when its gradients were not finite."""
    if loss_scale is not None:
        if isinstance(cfg, ScheduleConfig):
            ops.adam_ls(arena.data, arena.grad, arena.m, arena.v, cfg.lr, cfg.decay_steps, cfg.decay_rate,
                        cfg.staircase, cfg.beta_1, cfg.beta_2, cfg.epsilon, arena.iterations, loss_scale,
                        grad_scale=grad_scale)
        else:
            ops.adam_ls(arena.data, arena.grad, arena.m, arena.v, cfg.lr, 0, 1.0, False, cfg.beta_1, cfg.beta_2,
                        cfg.epsilon, arena.iterations, loss_scale, grad_scale=grad_scale)
        ops.counter_add_ls(arena.iterations, loss_scale)
        return
    if isinstance(cfg, ScheduleConfig):
        ops.adam_sched(arena.data, arena.grad, arena.m, arena.v, cfg.lr, cfg.decay_steps, cfg.decay_rate,
                       cfg.staircase, cfg.beta_1, cfg.beta_2, cfg.epsilon, arena.iterations, grad_scale=grad_scale)
    else:
        ops.adam(arena.data, arena.grad, arena.m, arena.v, cfg.lr, cfg.beta_1, cfg.beta_2, cfg.epsilon,
                 arena.iterations, grad_scale=grad_scale)
    ops.counter_add(arena.iterations, 1)


class VGGNetwork(GraphNetwork):
    """Frozen VGG19 feature extractor (block5_conv4).  ImageNet weights are a
    network download in the reference (keras.applications.VGG19(weights=
    "imagenet")); offline they load from a local .npz with Keras layer names
    (`vgg_weights`), else seeded He-normal weights stand in."""

    # fp16x3 from this many pixels per image: pix2pix's 256^2 and FastSRGAN's 512^2 gain, the
    # autoencoder's 64^2 VGG19 loses (bs4: 1036-1056 img/s vs 1074-1106 on bf16x6 / fp32 tiles) and
    # SRGAN's 96^2 is even (4172-4176 vs 4183-4185), profiles/r4/ab_x3_small_layers.txt.  A speed
    # rule only: one network planned on both sides of it holds weight planes per layout
    # (graph.GraphPlan, tests/test_mixed_math_gpu.py)
    X3_MIN_PIXELS = 128 * 128

    def __init__(self, weights=None, seed=4242, width=1, device=None):
        super().__init__(vgg19_features(width), seed=seed, device=device, kind="vgg19", trainable=False)
        # the frozen network's GEMMs on fp16x3 (include/dgan.h DG_MATH_F16X3: three fp16 piece
        # products, half the bf16x6 MFMA count) for large images when the library default is
        # bf16x6 (plan()); DG_VGG_MATH overrides (e.g. "bf16x6" for A/B runs)
        vm = os.environ.get("DG_VGG_MATH")
        self._auto_math = not vm and ops.default_conv_math() == ops.MATH_BF16X6
        if vm:
            self.conv_math = vm
        self.pretrained = False
        if weights:
            self.load_weights(weights)
            self.pretrained = True


    def plan(self, N, H, W, **kw):
        # (a math the owner set -- "fp16" under mixed_float16, sr_models -- stays)
        if self._auto_math and self.conv_math in (None, "f16x3"):
            self.conv_math = "f16x3" if H * W >= self.X3_MIN_PIXELS else None
        return super().plan(N, H, W, **kw)


class ContentLoss:
    """VGG19 content loss of one (gen, target) shape: value into a device
    scalar and, when requested, its gradient w.r.t. gen accumulated into a
    caller buffer (srgan.py:70-76, pix2pix.py:45-51).

    The two VGG19 calls (on G(x) and on the target) run as ONE forward over
    2N images (twice the GEMM rows per conv); the backward runs over the G(x)
    half only, on an N-image plan whose activations are views of the first
    half of the batched forward's buffers."""

    def __init__(self, vgg, N, H, W, device, train=True, split=False):
        """split: the target's VGG19 forward on its own N-image plan (forward_target, e.g. on a
        second stream beside the generator's forward, whose output it does not need) and G(x)'s
        on another; otherwise both in one 2N forward."""
        self.vgg = vgg
        self.N = N
        self.split = split
        e = lambda s: torch.empty(s, dtype=torch.float32, device=device)
        if split:
            self.fplan = vgg.plan(N, H, W, slots=1, train=False, param_grads=False)
            self.tplan = vgg.plan(N, H, W, slots=1, train=False, param_grads=False, tag="target")
            self.pre = e((N, H, W, 3))                    # pre(gen)
            self.pre_t = e((N, H, W, 3))                  # pre(target)
            self.tfeat = None
        else:
            self.fplan = vgg.plan(2 * N, H, W, slots=1, train=False, param_grads=False)
            self.tplan = None
            self.pre = e((2 * N, H, W, 3))                # [pre(gen); pre(target)]
        self.bplan = vgg.plan(N, H, W, slots=1, train=True, param_grads=False, alias=self.fplan) if train else None
        self.dpre = e((N, H, W, 3)) if train else None
        self.dfeat = e((N,) + tuple(self.fplan.out_shape[1:])) if train else None
        self.value = torch.zeros(1, dtype=torch.float32, device=device)
        self.ws_bytes = max(self.fplan.ws_bytes, self.bplan.ws_bytes if train else 0, ops.mse_workspace_bytes())
        self.tws_bytes = self.tplan.ws_bytes if split else 0

    def forward_target(self, tgt, ws=None):
        """(split) the target's features, read by the next forward()."""
        ops.vgg_preprocess_fwd(tgt, self.pre_t)
        self.tfeat = self.tplan.forward(self.pre_t, slot=0, training=False, ws=ws)
        return self.tfeat

    def feature_sources(self):
        """((plan, rows) of G(x)'s VGG19 forward, (plan, rows) of the target's): where the
        last step's activations of each live (one 2N plan, or the two N plans of split)."""
        N = self.N
        if self.split:
            return (self.fplan, slice(0, N)), (self.tplan, slice(0, N))
        return (self.fplan, slice(0, N)), (self.fplan, slice(N, 2 * N))

    def settled(self):
        """The shared frozen weight planes are split for the current VGG19 weights: the two
        plans may then run on two streams (the first forward after a weight change splits them,
        and the plans share the buffers -- that one runs in sequence)."""
        return getattr(self, "_settled", None) == getattr(self.vgg.arena, "version", 0)

    def mark_settled(self):
        self._settled = getattr(self.vgg.arena, "version", 0)

    def forward(self, gen, tgt, grad_weight=1.0, ws=None, tsync=None):
        """tsync (split): called before the target's features are read (a stream join)."""
        N = self.N
        if self.split:
            if self.tfeat is None:
                raise RuntimeError("ContentLoss(split=True): forward_target first")
            ops.vgg_preprocess_fwd(gen, self.pre)
            fg = self.fplan.forward(self.pre, slot=0, training=False, ws=ws)
            ft = self.tfeat
            if tsync is not None:
                tsync()
        else:
            ops.vgg_preprocess_fwd(gen, self.pre[:N])
            ops.vgg_preprocess_fwd(tgt, self.pre[N:])
            f = self.fplan.forward(self.pre, slot=0, training=False, ws=ws)
            fg, ft = f[:N], f[N:]
        # MeanSquaredError()(target_features, gen_features): grad w.r.t. gen features
        ops.mse(fg, ft, self.value, scale=FEAT_SCALE, da=self.dfeat, grad_weight=grad_weight, ws=ws)
        return self.value

    def backward(self, dgen, beta=1.0, ws=None):
        """dgen += d content / d gen (through VGG and preprocess_input)."""
        self.bplan.slots[0][self.vgg.graph.input.id] = self.pre[:self.N]
        self.bplan.backward(self.dfeat, slot=0, input_grad=self.dpre, input_beta=0.0, ws=ws, params=False)
        ops.vgg_preprocess_bwd(self.dpre, dgen, beta=beta)


# coefficient sets of dg_gan_loss: (w_adv, w_var, disc_scale, t_mae, t_mse, t_content, t_var)
COEF = {
    # train_srgan.py:87-96: gen = content + adv + 0*mse + mae + 0*var; disc = real + fake
    "srgan": (1e-3, 1e-5, 1.0, 1.0, 0.0, 1.0, 0.0),
    # train_fsrgan.py:88-96: gen = content + adv + 0*mse + mae; disc = 0.5*(valid + fake)
    "fsrgan": (1e-3, 1e-5, 0.5, 1.0, 0.0, 1.0, 0.0),
    # train_autoencoder.py:88-100: perceptual = content + adv + 0*mse + mae; disc = valid + fake
    "autoencoder": (1e-3, 1e-5, 1.0, 1.0, 0.0, 1.0, 0.0),
}


# the target's work (its VGG19 features and D(real)) on a second stream beside G's forward,
# which it does not need -- for outputs of >= 256^2 pixels: FastSRGAN 512^2 +1.7 %, while the
# 96^2 SRGAN (-2.5 %) and the 64^2 autoencoder (-7 %) lose more to the halved VGG19 batch than
# the overlap returns (profiles/r5/ab_sr_overlap.txt; DG_SR_NO_OVERLAP: never)
SR_OVERLAP = not os.environ.get("DG_SR_NO_OVERLAP")
SR_OVERLAP_MIN_PIXELS = 256 * 256

LOSS_SCALE_INIT = 2.0 ** 15     # tf.keras DynamicLossScale defaults (srgan.py:64-67)
LOSS_SCALE_PERIOD = 2000
LOSS_SCALE_MULT = 2.0


def new_loss_scale(device):
    """Device state of one dynamic loss scale: {scale, good steps, finite flag, 0}."""
    return torch.tensor([LOSS_SCALE_INIT, 0.0, 1.0, 0.0], dtype=torch.float32, device=device)


class SRTrainer:
    """Static plan of one SR-family training step for x [N,h,w,3] -> y [N,H,W,3].

    loss_scales: (G, D) device loss-scale states for the fp16 conv math (the
    reference's mixed_float16 policy with LossScaleOptimizer, train_srgan.py:
    98-109): the loss-gradient seeds are multiplied by the scale, so every fp16
    GEMM operand of the backward carries scaled gradients; the gradients are
    checked for inf / nan after the (all-reduced) backward and Adam unscales
    them or skips the step, then the scale is updated (Keras' dynamic rule)."""

    def __init__(self, G, D, vgg, N, in_hw, out_hw, device, coef, g_opt, d_opt, grad_sync=None, loss_scales=None):
        self.G, self.D, self.vgg = G, D, vgg
        self.N = N
        h, w = in_hw
        H, W = out_hw
        self.coef = tuple(coef)
        self.g_opt, self.d_opt = g_opt, d_opt
        self.grad_sync = grad_sync
        self.ls_g, self.ls_d = loss_scales if loss_scales is not None else (None, None)
        self.Gp = G.plan(N, h, w, slots=1, train=True)
        if tuple(self.Gp.out_shape) != (N, H, W, 3):
            raise ValueError(f"generator output {self.Gp.out_shape} != target {(N, H, W, 3)}")
        self.Dp = D.plan(N, H, W, slots=2, train=True)
        e = lambda s: torch.empty(s, dtype=torch.float32, device=device)
        ls = self.Dp.out_shape
        self.dzr, self.dzf_d, self.dzf_g = e(ls), e(ls), e(ls)
        self.dgen = e((N, H, W, 3))
        self.loss = torch.zeros(7, dtype=torch.float32, device=device)
        dev = torch.device(device)
        ov = SR_OVERLAP and dev.type == "cuda" and H * W >= SR_OVERLAP_MIN_PIXELS
        self.content = ContentLoss(vgg, N, H, W, device, split=ov) if vgg is not None else None
        wsb = [self.Gp.ws_bytes, self.Dp.ws_bytes, ops.gan_loss_workspace_bytes()]
        if self.content:
            wsb.append(self.content.ws_bytes)
        self.ws = ops.Workspace(device)
        self.ws.get(max(wsb))
        self.side = None
        if ov:
            self.side = torch.cuda.Stream(device=dev)
            self.ws_side = ops.Workspace(device)
            self.ws_side.get(max(self.Dp.ws_bytes, self.content.tws_bytes if self.content else 0))

    @property
    def gen_output(self):
        return self.Gp.slots[0][self.G.graph.output.id]

    def step(self, x, y, apply=True):
        """x [N,h,w,3], y [N,H,W,3] device fp32 in [-1, 1].  Returns the 7 loss
        values (gen_total, adv, mae, mse, content, disc, var) on the device."""
        x = x if x.is_contiguous() else x.contiguous()
        y = y if y.is_contiguous() else y.contiguous()
        ws = self.ws
        Gp, Dp = self.Gp, self.Dp
        # ---- forward (train_srgan.py:76-80) ---------------------------------
        # (the target's VGG19 features and D(real) beside G's forward once the frozen VGG19's
        # shared weight planes are settled; D(fake) follows D(real) on the joined stream -- the
        # two slots of D's plan share its per-plan state)
        main = torch.cuda.current_stream() if self.side is not None else None
        ov = (self.side is not None and not ops.profiling() and
              (self.content is None or self.content.settled()))
        zr = None
        if ov:
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                if self.content is not None:
                    self.content.forward_target(y, ws=self.ws_side)
                zr = Dp.forward(y, slot=0, training=True, ws=self.ws_side)
        elif self.content is not None and self.content.split:
            self.content.forward_target(y, ws=ws)
        gen = Gp.forward(x, slot=0, training=True, ws=ws)
        if ov:
            main.wait_stream(self.side)
        else:
            zr = Dp.forward(y, slot=0, training=True, ws=ws)
        zf = Dp.forward(gen, slot=1, training=True, ws=ws)
        content = None
        if self.content is not None:
            content = self.content.forward(gen, y, grad_weight=self.coef[5], ws=ws)
        # ---- losses and their gradients (train_srgan.py:84-96) -------------
        ops.gan_loss(gen, y, zr, zf, self.loss, self.coef, content=content, dgen=self.dgen, dlogit_real_d=self.dzr,
                     dlogit_fake_d=self.dzf_d, dlogit_fake_g=self.dzf_g, ws=ws)
        if self.ls_g is not None:
            # get_scaled_loss (train_srgan.py:98-100): the gradient seeds of each loss times its scale
            for t in (self.dzr, self.dzf_d):
                ops.scale_by(t, self.ls_d)
            for t in (self.dgen, self.dzf_g) + ((self.content.dfeat,) if self.content is not None else ()):
                ops.scale_by(t, self.ls_g)
        sync = self.grad_sync
        # ---- disc gradients (train_srgan.py:105-106) ------------------------
        Dp.backward(self.dzr, slot=0, param_beta=0.0, ws=ws)
        Dp.backward(self.dzf_d, slot=1, param_beta=1.0, ws=ws)
        if sync:
            sync.start("D")
        # ---- gen gradients: through D(fake) and VGG(G(x)) into G ------------
        Dp.backward(self.dzf_g, slot=1, params=False, input_grad=self.dgen, input_beta=1.0, ws=ws)
        if self.content is not None:
            self.content.backward(self.dgen, beta=1.0, ws=ws)
        Gp.backward(self.dgen, slot=0, param_beta=0.0, ws=ws,
                    on_grads_ready=(sync.ready_G if sync else None))
        if sync:
            sync.finish()
        if self.ls_g is not None:
            # LossScaleOptimizer.apply_gradients: are the (all-reduced) gradients finite?
            # The flag is re-armed here, so a step(apply=False) that saw inf / nan (and ran
            # no loss_scale_update) does not leave it set for the next step.
            ops.fill(self.ls_g[2:3], 1.0)
            ops.fill(self.ls_d[2:3], 1.0)
            ops.check_finite(self.G.arena.grad, self.ls_g)
            ops.check_finite(self.D.arena.grad, self.ls_d)
        # ---- apply_gradients (train_srgan.py:113-114) -----------------------
        if self.content is not None and self.content.split:
            self.content.mark_settled()
        if apply:
            scale = sync.grad_scale if sync else 1.0
            apply_adam(self.G.arena, self.g_opt, scale, self.ls_g)
            apply_adam(self.D.arena, self.d_opt, scale, self.ls_d)
            if self.ls_g is not None:
                ops.loss_scale_update(self.ls_g, LOSS_SCALE_PERIOD, LOSS_SCALE_MULT)
                ops.loss_scale_update(self.ls_d, LOSS_SCALE_PERIOD, LOSS_SCALE_MULT)
        return self.loss
