"""Network definitions of the SRGAN, FastSRGAN and Autoencoder families and
the VGG19 feature extractor, as dgan.graph Graphs.

Each builder follows the reference's Keras model function layer by layer
(file:line cited per builder); activations that directly follow a Conv2D or a
BatchNormalization are fused into that node.  Variable names are
"<layer>/<kernel|bias|gamma|beta|alpha|depthwise_kernel>" with Keras-style
layer names.
"""
from .graph import Graph

W_INIT = ("normal", 0.0, 0.02)   # tf.random_normal_initializer(0., 0.02)   (srgan.py:130)
G_INIT = ("normal", 1.0, 0.02)   # tf.random_normal_initializer(1., 0.02)   (srgan.py:131)


def srgan_generator(scale=4, n_blocks=16, gf=64):
    """SRGAN.build_generator (srgan.py:129-185)."""
    g = Graph("generator")
    x = g.input
    n = g.conv(x, gf, 3, use_bias=False, kernel_init=W_INIT, name="conv2d")                 # :158
    n = g.bn(n, gamma_init=G_INIT, name="batch_normalization")                               # :159
    n = g.prelu(n, name="p_re_lu")                                                           # :161
    temp = n
    for i in range(n_blocks):                                                                # :165-175
        nn = g.conv(n, gf, 3, use_bias=False, kernel_init=W_INIT, name=f"block_{i}_conv1")
        nn = g.bn(nn, gamma_init=G_INIT, act="relu", name=f"block_{i}_bn1")
        nn = g.conv(nn, gf, 3, use_bias=False, kernel_init=W_INIT, name=f"block_{i}_conv2")
        nn = g.bn(nn, gamma_init=G_INIT, name=f"block_{i}_bn2")
        n = g.add(n, nn, name=f"block_{i}_add")
    n = g.conv(n, gf, 3, use_bias=False, kernel_init=W_INIT, name="conv2d_post")             # :177
    n = g.bn(n, gamma_init=G_INIT, name="batch_normalization_post")                          # :178
    n = g.add(n, temp, name="add_long")                                                      # :180
    for i in range(scale // 2):                                                              # :184-185
        n = g.conv(n, 256, 3, use_bias=True, kernel_init=W_INIT, name=f"deconv_{i}_conv")    # :146
        n = g.prelu(n, block=2, name=f"deconv_{i}_p_re_lu")                                  # :147-148
    out = g.conv(n, 3, 1, use_bias=True, kernel_init=W_INIT, act="tanh", name="conv2d_out")  # :187-188
    return g.set_output(out)


def sr_discriminator(df=32, name="discriminator"):
    """The Fast-SRGAN-style discriminator shared by SRGAN.build_discriminator
    (srgan.py:232-272), FastSRGAN.build_discriminator (fsrgan.py:216-258) and,
    with a sigmoid output, Autoencoder.build_discriminator (autoencoder.py:188-229):
    8 x [Conv3 (+bias, glorot) -> BN(momentum .8) -> LeakyReLU(.2)] -> Conv1x1(1)."""
    g = Graph(name)
    h = g.input
    spec = [(df, 1, False), (df, 2, True), (df, 1, True), (df, 2, True),
            (df * 2, 1, True), (df * 2, 2, True), (df * 2, 1, True), (df * 2, 2, True)]
    for i, (f, s, bn) in enumerate(spec):
        if bn:
            h = g.conv(h, f, 3, strides=s, use_bias=True, name=f"d{i + 1}_conv")
            h = g.bn(h, momentum=0.8, act="lrelu", alpha=0.2, name=f"d{i + 1}_bn")
        else:
            h = g.conv(h, f, 3, strides=s, use_bias=True, act="lrelu", alpha=0.2, name=f"d{i + 1}_conv")
    out = g.conv(h, 1, 1, use_bias=True, name="logits")
    return g.set_output(out)


def _make_divisible(v, divisor, min_value=None):
    """fsrgan.py:103-110."""
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


def fsrgan_generator(gf=32, n_blocks=6, expansion=6):
    """FastSRGAN.build_generator (fsrgan.py:99-220): MobileNetV2 inverted
    residual blocks, then two pixel-shuffle x2 upsamplers."""
    g = Graph("generator")
    x = g.input
    c1 = g.conv(x, gf, 3, use_bias=True, name="conv2d")                                     # :198
    c1 = g.bn(c1, name="batch_normalization")                                                 # :199
    c1 = g.prelu(c1, name="p_re_lu")                                                          # :200

    def residual_block(inputs, filters, block_id):                                            # :112-177
        in_ch = inputs.C
        pw = _make_divisible(int(filters * 1.0), 8)
        h = inputs
        prefix = f"block_{block_id}_"
        if block_id:
            h = g.conv(h, expansion * in_ch, 1, use_bias=True, name=prefix + "expand")
            h = g.bn(h, epsilon=1e-3, momentum=0.999, act="relu", name=prefix + "expand_BN")
        else:
            prefix = "expanded_conv_"
        h = g.dwconv(h, use_bias=True, name=prefix + "depthwise")
        h = g.bn(h, epsilon=1e-3, momentum=0.999, act="relu", name=prefix + "depthwise_BN")
        h = g.conv(h, pw, 1, use_bias=True, name=prefix + "project")
        h = g.bn(h, epsilon=1e-3, momentum=0.999, name=prefix + "project_BN")
        if in_ch == pw:
            return g.add(inputs, h, name=prefix + "add")
        return h

    r = residual_block(c1, gf, 0)                                                             # :203-205
    for idx in range(1, n_blocks):
        r = residual_block(r, gf, idx)
    c2 = g.conv(r, gf, 3, use_bias=True, name="conv2d_post")                                  # :208
    c2 = g.bn(c2, name="batch_normalization_post")                                           # :209
    c2 = g.add(c2, c1, name="add_long")                                                       # :210
    u = c2
    for i in range(2):                                                                        # :213-214 (deconv2d :187-190)
        u = g.conv(u, gf * 4, 3, use_bias=True, name=f"deconv_{i}_conv")
        u = g.prelu(u, block=2, name=f"deconv_{i}_p_re_lu")
    out = g.conv(u, 3, 3, use_bias=True, act="tanh", name="conv2d_out")                       # :217-218
    return g.set_output(out)


def autoencoder_generator():
    """Autoencoder.build_autoencoder (autoencoder.py:89-185): a 5-level
    conv/maxpool encoder and a nearest-upsample + concat decoder."""
    g = Graph("Autoencoder")
    img = g.input

    def c(h, f, name, relu=True):                                                             # :91-108
        if relu:
            return g.conv(h, f, 3, use_bias=True, act="relu", kernel_init=("he_normal",), name=name)
        return g.conv(h, f, 3, use_bias=True, act="tanh", kernel_init=("lecun_normal",), name=name)

    h = c(img, 32, "conv1")
    h = c(h, 32, "conv1b")
    pool1 = g.maxpool(h, name="pool1")
    h = c(pool1, 44, "conv2")
    pool2 = g.maxpool(h, name="pool2")
    h = c(pool2, 56, "conv3")
    pool3 = g.maxpool(h, name="pool3")
    h = c(pool3, 76, "conv4")
    pool4 = g.maxpool(h, name="pool4")
    h = c(pool4, 100, "conv5")
    pool5 = g.maxpool(h, name="pool5")
    for k, (skip, f) in enumerate([(pool4, 152), (pool3, 112), (pool2, 84), (pool1, 64)]):   # :160-174
        lvl = 6 + k
        up = g.upsample_relu(pool5 if k == 0 else h, name=f"unpool{4 - k}")
        h = g.concat(up, skip, name=f"upconcat{4 - k}")
        h = c(h, f, f"conv{lvl}")
        h = c(h, f, f"conv{lvl}b")
    up = g.upsample_relu(h, name="unpool0")                                                   # :176
    h = g.concat(up, img, name="upconcat0")
    h = c(h, 64, "conv10")
    h = c(h, 32, "conv10b")
    out = c(h, 3, "conv11", relu=False)                                                       # :180
    return g.set_output(out)


VGG19_BLOCKS = [(64, 2), (128, 2), (256, 4), (512, 4), (512, 4)]


def vgg19_features(width=1):
    """keras.applications.VGG19(include_top=False) truncated at block5_conv4
    (post-ReLU), the content-loss feature extractor of every model
    (pix2pix.py:53-67, srgan.py:78-94).  `width` divides the channel counts
    (test-only)."""
    g = Graph("vgg19")
    h = g.input
    for b, (f, n) in enumerate(VGG19_BLOCKS):
        f = max(1, f // width)
        for i in range(n):
            h = g.conv(h, f, 3, use_bias=True, act="relu", kernel_init=("he_normal_plain",),
                       name=f"block{b + 1}_conv{i + 1}")
        if b < 4:
            h = g.maxpool(h, name=f"block{b + 1}_pool")
    return g.set_output(h)
