"""FastSRGAN model container — drop-in for the reference's fsrgan.py.

`FastSRGAN(args)` keeps the surface of fsrgan.py:5-72 (dgan.sr_models); the
MobileNetV2-style generator (fsrgan.py:99-214: 6 inverted residual blocks
with depthwise 3x3 convs, two pixel-shuffle x2 upsamplers) and the
discriminator (fsrgan.py:216-258) run as dgan.graph networks on libdgan.
The generator always upsamples x4 (two deconv2d, fsrgan.py:217-218).
"""
from dgan import zoo
from dgan.sr_models import DiscriminatorNet, SRFamily, sr_generator_net


class FastSRGAN(SRFamily):
    """SRGAN for fast super resolution."""
    kind = "fsrgan"
    coef_key = "fsrgan"

    def __init__(self, args):
        self.n_residual_blocks = 6
        self.gf = 32
        self.df = 32
        super().__init__(args)
        patch = int(self.hr_height / 2 ** 4)
        self.disc_patch = (patch, patch, 1)

    def build_networks(self, args):
        g = sr_generator_net(zoo.fsrgan_generator(gf=self.gf, n_blocks=self.n_residual_blocks), self.seed,
                             self.device)
        d = DiscriminatorNet(zoo.sr_discriminator(df=self.df), self.seed + 1, self.device)
        return g, d

    def build_generator(self):
        return self.generator

    def build_discriminator(self):
        return self.discriminator

    def trainer(self, x_shape, y_shape=None):
        if y_shape is None:
            y_shape = (x_shape[0], x_shape[1] * 4, x_shape[2] * 4, 3)
        return super().trainer(x_shape, y_shape)
