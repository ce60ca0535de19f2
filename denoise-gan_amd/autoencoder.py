"""Denoising Autoencoder container — drop-in for the reference's autoencoder.py.

`Autoencoder(args)` keeps the surface of autoencoder.py:4-62 (dgan.sr_models);
the U-shaped conv / maxpool / nearest-upsample + concat generator
(autoencoder.py:89-185) and the sigmoid-output discriminator
(autoencoder.py:188-229) run as dgan.graph networks on libdgan.  The
discriminator's call returns probabilities; training computes the
probability BCE from the pre-sigmoid logits, as Keras' binary_crossentropy
does when its input is a Sigmoid op (graph mode, train_autoencoder.py:66).
"""
from dgan import zoo
from dgan.sr_models import DiscriminatorNet, SRFamily, sr_generator_net


class Autoencoder(SRFamily):
    """ Denoising Autoencoder """
    kind = "autoencoder"
    coef_key = "autoencoder"

    def __init__(self, args):
        self.gf = 32
        self.df = 32
        super().__init__(args)
        # the AE maps H x W -> H x W (autoencoder.py:16-19: no downscale)
        self.scale = 1
        self.lr_height, self.lr_width = self.hr_height, self.hr_width
        self.lr_shape = (self.lr_height, self.lr_width, 3)
        self.hr_shape = (self.hr_height, self.hr_width, 3)
        patch = int(self.hr_height / 2 ** 4)
        self.disc_patch = (patch, patch, 1)

    def build_networks(self, args):
        if self.hr_height % 32 or self.hr_width % 32:
            raise ValueError("the autoencoder needs crop sizes divisible by 32 (five 2x2 pools)")
        g = sr_generator_net(zoo.autoencoder_generator(), self.seed, self.device)
        d = DiscriminatorNet(zoo.sr_discriminator(df=self.df, name="Discriminator"), self.seed + 1, self.device,
                             output_act="sigmoid")
        return g, d

    def build_autoencoder(self, name="Autoencoder"):
        return self.generator

    def build_discriminator(self, name="Discriminator"):
        return self.discriminator

    def trainer(self, x_shape, y_shape=None):
        return super().trainer(x_shape, y_shape or x_shape)
