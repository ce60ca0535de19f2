"""Pix2Pix model container — drop-in for the reference's pix2pix.py.

Same constructor and attribute surface as `Pix2Pix(args)` in
/root/reference/pix2pix.py:4-226, so train_pix2pix.py-style drivers keep
working; underneath, every layer runs on libdgan (hand-written gfx950 HIP)
through dgan.nets' static executors.

Reference surface kept:
  Pix2Pix(args)                      reads args.crop_size, args.retrain (pix2pix.py:15, :23)
  .hr_height/.hr_width/.lr_shape/.hr_shape, .iterations, .epochs, .retrain
  .gen_loss_object / .disc_loss_object   (:26-27; MSE and BCE-from-logits on the HIP path)
  .gen_optimizer / .disc_optimizer   Adam(2e-4, beta_1=0.5)            (:30-31)
  .gf / .df                           32 (unused by the reference too) (:39-40)
  .generator / .discriminator         networks                        (:43, build_gan :106-226)
  .content_loss(target, gen)          VGG19 content loss              (:45-51)  [see below]
  .generator_loss(d_fake, gen, tgt)   7-tuple                          (:74-94)
  .discriminator_loss(real, fake)     scalar                           (:96-103)

Differences that cannot be avoided offline (documented in DESIGN.md):
  * VGG19 ImageNet weights (pix2pix.py:59) are a network download.  `.vgg`
    is the same VGG19-to-block5_conv4 network on libdgan; it loads local
    weights from args.vgg_weights (.npz, Keras layer names) when given, else
    seeded He-normal stand-in weights.  args.content_loss=0 drops the term.
  * Dropout masks come from a counter-based hash (reproducible on the CPU
    oracle) instead of TF's RNG stream.
Extra (MI355X-specific) knobs, read from args when present:
  args.width (test-only channel divisor, default 1), args.seed,
  args.dropout_seed, args.identity_loss (default 1), args.content_loss
  (default 1), args.vgg_weights, args.vgg_width (test-only).
"""
import torch

from dgan import ops
from dgan.models import Adam, Discriminator, Generator, default_device, to_device
from dgan.trainer import Pix2PixTrainer
from dgan.sr_trainer import ContentLoss, VGGNetwork


class _MSE:
    """tf.keras.losses.MeanSquaredError() (mean over all elements), on the HIP loss kernel."""

    def __call__(self, y_true, y_pred):
        y_pred = to_device(y_pred, default_device())
        y_true = to_device(y_true, y_pred.device)
        z = torch.zeros(1, dtype=torch.float32, device=y_pred.device)
        out = torch.empty(8, dtype=torch.float32, device=y_pred.device)
        ops.p2p_loss(y_pred, y_true, z, z, out, weights=(0.0, 0.0, 1.0, 0.0, 0.0, 0.0))
        return out[3]


class _BCELogits:
    """tf.keras.losses.BinaryCrossentropy(from_logits=True) marker; the HIP loss kernel implements it."""
    from_logits = True


class Pix2Pix(object):
    """ Denoising Pix2Pix """

    def __init__(self, args):
        self.hr_height = args.crop_size
        self.hr_width = args.crop_size
        self.lr_height = self.hr_height
        self.lr_width = self.hr_width
        self.lr_shape = (self.lr_height, self.lr_width, 3)
        self.hr_shape = (self.hr_height, self.hr_width, 3)
        self.iterations = 0
        self.epochs = 0
        self.retrain = bool(getattr(args, "retrain", False))
        self.fp16 = bool(getattr(args, "fp16", False))
        self.device = default_device()

        self.gen_loss_object = _MSE()
        self.disc_loss_object = _BCELogits()

        self.gen_optimizer = Adam(2e-4, beta_1=0.5)
        self.disc_optimizer = Adam(2e-4, beta_1=0.5)


        self.gf = 32
        self.df = 32

        self.width = int(getattr(args, "width", 1))
        self.seed = int(getattr(args, "seed", 1234))
        self.dropout_seed = int(getattr(args, "dropout_seed", 0))
        self.identity = bool(int(getattr(args, "identity_loss", 1)))
        self.dropout_rate = float(getattr(args, "dropout_rate", 0.5))
        self.loss_weights = tuple(getattr(args, "loss_weights", ops.LOSS_WEIGHTS_REF))
        self.use_content = bool(int(getattr(args, "content_loss", 1)))
        if not self.use_content:
            self.loss_weights = self.loss_weights[:5] + (0.0,)
        # VGG19(weights="imagenet") (pix2pix.py:53-67) is a remote download: local .npz or seeded stand-in
        self.vgg = VGGNetwork(weights=getattr(args, "vgg_weights", None), seed=self.seed + 7,
                              width=int(getattr(args, "vgg_width", 1)), device=self.device) if self.use_content else None
        self._content = {}
        self._ws = None
        self.generator, self.discriminator = self.build_gan()
        self.gen_optimizer.bind(self.generator.arena)
        self.disc_optimizer.bind(self.discriminator.arena)
        self._trainers = {}
        self.grad_sync = None  # set by dgan.dist for data-parallel runs

    # ------------------------------------------------------------------
    def content_loss(self, target, gen_output):
        """MSE(vgg(pre(target))/12.75, vgg(pre(gen))/12.75) (pix2pix.py:45-51)."""
        if self.vgg is None:
            return torch.zeros((), dtype=torch.float32, device=self.device)
        tgt, gen = to_device(target, self.device), to_device(gen_output, self.device)
        N, H, W, _ = gen.shape
        if (N, H, W) not in self._content:
            self._content[(N, H, W)] = ContentLoss(self.vgg, N, H, W, self.device, train=False)
        c = self._content[(N, H, W)]
        return c.forward(gen, tgt, ws=self._workspace(c.ws_bytes))[0].clone()

    def _workspace(self, nbytes):
        """One workspace for the eager Keras-surface calls (grown on demand, never per call)."""
        if self._ws is None:
            self._ws = ops.Workspace(self.device)
        self._ws.get(nbytes)
        return self._ws

    def build_vgg(self):
        return self.vgg

    def _loss_values(self, gen, tgt, ident, real, fake):
        out = torch.empty(8, dtype=torch.float32, device=self.device)
        gen, tgt = to_device(gen, self.device), to_device(tgt, self.device)
        real, fake = to_device(real, self.device), to_device(fake, self.device)
        cont = self.content_loss(tgt, gen).reshape(1) if self.vgg is not None else None
        ops.p2p_loss(gen, tgt, real, fake, out, ident=None if ident is None else to_device(ident, self.device),
                     weights=self.loss_weights, content=cont)
        return out

    def generator_loss(self, disc_generated_output, gen_output, target):
        """7-tuple (total, gan, l1, l2, content, var, identity) (pix2pix.py:74-94).
        Runs the identity pass G(target, training=True) like the reference (:90)."""
        ident = self.generator(target, training=True) if self.identity else None
        o = self._loss_values(gen_output, target, ident, disc_generated_output, disc_generated_output)
        return o[0], o[1], o[2], o[3], o[4], o[6], o[7]

    def discriminator_loss(self, disc_real_output, disc_generated_output):
        """BCE(1, real) + BCE(0, fake) (pix2pix.py:96-103)."""
        z = torch.zeros((1, 1, 1, 3), dtype=torch.float32, device=self.device)
        return self._loss_values(z, z, None, disc_real_output, disc_generated_output)[5]

    def build_gan(self, name="Pix2Pix"):
        generator = Generator(width=self.width, seed=self.seed, device=self.device)
        discriminator = Discriminator(width=self.width, seed=self.seed + 1, device=self.device)
        return generator, discriminator

    # ------------------------------------------------------------------
    def trainer(self, shape):
        N, H, W = int(shape[0]), int(shape[1]), int(shape[2])
        key = (N, H, W)
        if key not in self._trainers:
            self._trainers[key] = Pix2PixTrainer(
                self.generator.arena, self.generator.bn, self.discriminator.arena, self.discriminator.bn, N, H, W,
                self.device, width=self.width, identity=self.identity, loss_weights=self.loss_weights,
                drop_rate=self.dropout_rate, drop_seed=self.dropout_seed, g_opt=self.gen_optimizer,
                d_opt=self.disc_optimizer, grad_sync=self.grad_sync, vgg=self.vgg)
        return self._trainers[key]
