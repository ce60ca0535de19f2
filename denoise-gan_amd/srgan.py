"""SRGAN model container — drop-in for the reference's srgan.py.

`SRGAN(args)` keeps the constructor and attribute surface of srgan.py:7-66
(see dgan.sr_models); the generator (srgan.py:129-188: conv-BN-PReLU, 16
residual blocks, scale//2 pixel-shuffle x2 upsamplers, 1x1 conv + tanh) and
the discriminator (srgan.py:232-272) run as dgan.graph networks on libdgan.
`generator_loss` / `discriminator_loss` follow srgan.py:97-126.
"""
from dgan import ops, zoo
from dgan.models import to_device
from dgan.sr_models import DiscriminatorNet, SRFamily, sr_generator_net

import torch


class SRGAN(SRFamily):
    """SRGAN for fast super resolution."""
    kind = "srgan"
    coef_key = "srgan"

    def build_networks(self, args):
        g = sr_generator_net(zoo.srgan_generator(scale=self.scale), self.seed, self.device)
        d = DiscriminatorNet(zoo.sr_discriminator(df=32), self.seed + 1, self.device)
        return g, d

    def build_generator(self):
        return self.generator

    def build_discriminator(self):
        return self.discriminator

    def _losses(self, disc_generated_output, gen_output, target, disc_real_output=None, coef=None):
        gen, tgt = to_device(gen_output, self.device), to_device(target, self.device)
        fake = to_device(disc_generated_output, self.device)
        real = fake if disc_real_output is None else to_device(disc_real_output, self.device)
        cont = self.content_loss(tgt, gen).reshape(1)
        out = torch.empty(7, dtype=torch.float32, device=self.device)
        ops.gan_loss(gen, tgt, real, fake, out, coef, content=cont)
        return out

    def generator_loss(self, disc_generated_output, gen_output, target):
        """(total, adv, l1, l2, cont, var) with total = adv + l2 + cont (srgan.py:97-120)."""
        o = self._losses(disc_generated_output, gen_output, target, coef=(1e-3, 1e-5, 1.0, 0.0, 1.0, 1.0, 0.0))
        return o[0], o[1], o[2], o[3], o[4], o[6]

    def discriminator_loss(self, disc_real_output, disc_generated_output):
        """BCE(1, real) + BCE(0, fake) (srgan.py:122-127)."""
        z = torch.zeros((1, 1, 1, 3), dtype=torch.float32, device=self.device)
        real = to_device(disc_real_output, self.device)
        fake = to_device(disc_generated_output, self.device)
        out = torch.empty(7, dtype=torch.float32, device=self.device)
        ops.gan_loss(z, z, real, fake, out, (1e-3, 1e-5, 1.0, 0.0, 0.0, 0.0, 0.0))
        return out[5]
