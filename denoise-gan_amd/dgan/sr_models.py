"""Model containers of the SR family (SRGAN, FastSRGAN, Autoencoder) with
the reference's constructor / attribute surface (srgan.py:7-66,
fsrgan.py:5-72, autoencoder.py:4-62), on dgan.graph networks.

Reference surface kept:
  Model(args)  reads args.scale, args.crop_size, args.fp16, args.lr (+ args.retrain for the AE)
  .scale .hr_height .hr_width .lr_height .lr_width .lr_shape .hr_shape .iterations .epochs .fp16
  .gen_schedule / .disc_schedule     ExponentialDecay(lr, 100000, 0.1, staircase), TTUR lr*5
  .gen_optimizer / .disc_optimizer   Adam(learning_rate=schedule)  (+ the LossScaleOptimizer
                                     get_scaled_loss / get_unscaled_gradients surface)
  .vgg                               frozen VGG19 to block5_conv4
  .generator / .discriminator        Keras-shaped networks (call, trainable_variables, save, ...)
  .content_loss(hr, sr)              VGG feature MSE / 12.75^2
  .disc_patch / .gf / .df / .n_residual_blocks where the reference defines them

mixed_float16 (args.fp16, srgan.py:63-66, train_srgan.py:312-318): every
eligible conv GEMM of G, D and VGG19 rounds its operands to fp16 and runs
one fp16 MFMA per product (include/dgan.h DG_MATH_FP16; activations,
accumulation and the layer math stay fp32), and both optimizers carry a
dynamic loss scale (2^15, halve and skip on inf/nan, double after 2000
finite steps) on the device.  Without args.fp16 the conv GEMMs are
fp32-accurate (bf16x6) and the loss scale is 1.
"""
import torch

from . import ops
from .graph import GraphNetwork
from .models import Adam, default_device, to_device
from .sr_trainer import COEF, ScheduleConfig, SRTrainer, VGGNetwork, ContentLoss
from . import zoo

ExponentialDecay = ScheduleConfig


class _LossScaleAdam(Adam):
    """Adam + the mixed_precision.LossScaleOptimizer surface used by train_srgan.py:98-109.
    With args.fp16 the scale is the trainer's device state (dynamic, 2^15 initial);
    otherwise it is 1 (fp32-accurate conv math needs none)."""

    _ls = None   # device loss-scale state (dgan.sr_trainer.new_loss_scale), fp16 only

    @property
    def loss_scale(self):
        return float(self._ls[0].item()) if self._ls is not None else 1.0

    def get_scaled_loss(self, loss):
        return loss * self.loss_scale

    def get_unscaled_gradients(self, grads):
        s = self.loss_scale
        return [None if g is None else g / s for g in grads]


class SRFamily(object):
    kind = "sr"
    coef_key = "srgan"

    def __init__(self, args):
        self.scale = int(getattr(args, "scale", 1))
        self.hr_height = int(args.crop_size)
        self.hr_width = int(args.crop_size)
        self.lr_height = self.hr_height // self.scale
        self.lr_width = self.hr_width // self.scale
        self.lr_shape = [self.lr_height, self.lr_width, 3]
        self.hr_shape = [self.hr_height, self.hr_width, 3]
        self.iterations = 0
        self.epochs = 0
        self.fp16 = bool(getattr(args, "fp16", False))
        self.retrain = bool(getattr(args, "retrain", False))
        self.device = default_device()
        lr = float(getattr(args, "lr", 1e-3))
        self.gen_schedule = ExponentialDecay(lr, decay_steps=100000, decay_rate=0.1, staircase=True)
        self.disc_schedule = ExponentialDecay(lr * 5, decay_steps=100000, decay_rate=0.1, staircase=True)
        self.gen_optimizer = _LossScaleAdam(learning_rate=self.gen_schedule)
        self.disc_optimizer = _LossScaleAdam(learning_rate=self.disc_schedule)
        self.seed = int(getattr(args, "seed", 1234))
        self.use_content = bool(int(getattr(args, "content_loss", 1)))
        vw = getattr(args, "vgg_weights", None)
        self.vgg = VGGNetwork(weights=vw, seed=self.seed + 7, width=int(getattr(args, "vgg_width", 1)),
                              device=self.device) if self.use_content else None
        self.generator, self.discriminator = self.build_networks(args)
        self.loss_scales = None
        if self.fp16:
            from .sr_trainer import new_loss_scale
            for net in (self.generator, self.discriminator, self.vgg):
                if net is not None:
                    net.conv_math = "fp16"
            self.loss_scales = (new_loss_scale(self.device), new_loss_scale(self.device))
            self.gen_optimizer._ls, self.disc_optimizer._ls = self.loss_scales
        self.gen_optimizer.bind(self.generator.arena)
        self.disc_optimizer.bind(self.discriminator.arena)
        self.coef = COEF[self.coef_key]
        self._trainers = {}
        self._content = {}
        self._ws = None
        self.grad_sync = None

    # --- to override -----------------------------------------------------
    def build_networks(self, args):
        raise NotImplementedError

    # --- reference methods ------------------------------------------------
    def build_vgg(self):
        return self.vgg

    def content_loss(self, hr, sr):
        """MeanSquaredError()(vgg(pre(hr))/12.75, vgg(pre(sr))/12.75) (srgan.py:69-76)."""
        if self.vgg is None:
            return torch.zeros((), dtype=torch.float32, device=self.device)
        hr, sr = to_device(hr, self.device), to_device(sr, self.device)
        N, H, W, _ = sr.shape
        key = (N, H, W)
        if key not in self._content:
            self._content[key] = ContentLoss(self.vgg, N, H, W, self.device, train=False)
        c = self._content[key]
        if self._ws is None:
            self._ws = ops.Workspace(self.device)
        self._ws.get(c.ws_bytes)
        return c.forward(sr, hr, ws=self._ws)[0].clone()

    def _sched(self, opt):
        s = opt.learning_rate
        if isinstance(s, ScheduleConfig):
            return ScheduleConfig(s.lr, s.decay_steps, s.decay_rate, s.staircase, opt.beta_1, opt.beta_2,
                                  opt.epsilon)
        return ScheduleConfig(float(s), 0, 1.0, False, opt.beta_1, opt.beta_2, opt.epsilon)

    def trainer(self, x_shape, y_shape=None):
        N, h, w = int(x_shape[0]), int(x_shape[1]), int(x_shape[2])
        if y_shape is None:
            H, W = h * self.scale, w * self.scale
        else:
            H, W = int(y_shape[1]), int(y_shape[2])
        key = (N, h, w, H, W)
        if key not in self._trainers:
            self._trainers[key] = SRTrainer(self.generator, self.discriminator, self.vgg, N, (h, w), (H, W),
                                            self.device, self.coef, self._sched(self.gen_optimizer),
                                            self._sched(self.disc_optimizer), grad_sync=self.grad_sync,
                                            loss_scales=self.loss_scales)
        return self._trainers[key]


class DiscriminatorNet(GraphNetwork):
    """Discriminator whose call returns `output_act(logits)`; training uses the
    logits directly (Keras' binary_crossentropy recovers them from a Sigmoid
    op in graph mode)."""

    def __init__(self, graph, seed, device, output_act=None):
        super().__init__(graph, seed=seed, device=device, kind="discriminator")
        self.output_act = output_act

    def __call__(self, x, training=False):
        y = super().__call__(x, training=training)
        if self.output_act:
            ops.act_fwd(y, y, self.output_act)
        return y


def sr_generator_net(graph, seed, device):
    return GraphNetwork(graph, seed=seed, device=device, kind="generator")
