"""pix2pix training driver — drop-in for the reference's train_pix2pix.py.

`train_step(model, x, y)` keeps the reference signature and 8-tuple return
(train_pix2pix.py:33-71); it runs the whole step (G/D forwards, losses, both
gradients, Adam G then D) as one fused launch sequence on libdgan.  `train`
and `main` follow :73-107 and :112-195 (TensorBoard -> dgan.summary JSONL,
tf.train.Checkpoint -> dgan.checkpoint, .h5 -> .npz; the shared loop is
dgan.driver.run).  The published driver crashes before training (`policy`
undefined at :231 when fp16=0, and DataLoader needs args.scale /
args.jpeg_quality absent from `params`); this one supplies
scale=1 and jpeg_quality=50.  Steps per epoch = images // batch_size
(DataLoader, drop_remainder); --synthetic 1 trains on seeded synthetic
pairs instead of image_dir.
"""
import os
from argparse import ArgumentParser

import numpy as np
import torch

from dataloader import DataLoader
from pix2pix import Pix2Pix
from dgan import driver
from dgan.models import to_device


def train_step(model, x, y):
    """Single pix2pix step.  x: noisy batch, y: clean batch (NHWC, [-1, 1]).
    Returns (gen_total, gen_gan, gen_l1, gen_l2, content, disc, var, identity)
    as device scalars (no host synchronisation)."""
    x = to_device(x, model.device)
    y = to_device(y, model.device)
    loss = model.trainer(x.shape).step(x, y)
    return tuple(loss[i] for i in range(8))


def train(model, dataset, args, writer):
    log_iter = args.save_iter
    with writer.as_default():
        for x, y in dataset:
            losses = train_step(model, x, y)
            model.iterations += 1
            if model.iterations % log_iter == 0:
                vals = torch.stack(losses).cpu().numpy()
                names = ["Generator Losses/gen_total_loss", "Generator Losses/gen_gan_loss",
                         "Generator Losses/gen_l1_loss", "Generator Losses/gen_l2_loss",
                         "Generator Losses/content_loss", "Discriminator Losses/disc_loss",
                         "Generator Losses/total_variation", "Generator Losses/identity_loss"]
                for n, v in zip(names, vals):
                    writer.scalar(n, v, step=model.epochs + 1)
                gen = model.generator(x, training=False)
                writer.image("Images/Generated", (255 * (gen.cpu().numpy() + 1) / 2).astype(np.uint8),
                             step=model.epochs + 1)
                writer.flush()


def get_path(path):
    return os.path.realpath(os.path.expanduser(os.path.expandvars(path)))


def save_final(model, timestamp):
    """Final exports (train_pix2pix.py:189-195; .h5 -> .npz + .json)."""
    model.generator.save(os.path.join(model.model_dir, "pix2pix.npz"))
    model.discriminator.save(os.path.join(model.model_dir, "discriminator_p2p.npz"))
    model.generator.save(os.path.join(model.model_dir, "backups", f"pix2pix_{timestamp}.npz"))
    model.discriminator.save(os.path.join(model.model_dir, "backups", f"discriminator_p2p_{timestamp}.npz"))


def main(args):
    """train_pix2pix.py:112-195 (dgan.driver.run: restore, epochs, checkpoints, exports)."""
    ds = DataLoader(args).dataset()
    if args.save_iter > len(ds):
        args.save_iter = max(1, len(ds))
    model = Pix2Pix(args)
    model.model_dir = args.model_dir
    return driver.run(args, model, ds, train, save_final)


params = dict(
    image_dir=get_path("~/Data/DIV2K/DIV2K_train_HR"),
    batch_size=1,
    epochs=1,
    crop_size=256,
    lr=1e-3,
    save_iter=200,
    model_dir=get_path("./models"),
    logdir=get_path("./logs"),
    retrain=0,
    save_model=1,
    ckpt=1,
    fp16=0,
    scale=1,
    jpeg_quality=50,
    synthetic=0,
    steps_per_epoch=8,   # synthetic pairs only; image_dir runs use images // batch_size
    seed=0,
)


def parse_args(argv=None):
    parser = ArgumentParser()
    for key, value in params.items():
        parser.add_argument("--" + key, default=value, type=type(value))
    args = parser.parse_args(argv)
    args.retrain = bool(args.retrain)
    args.save_model = bool(args.save_model)
    args.ckpt = bool(args.ckpt)
    args.fp16 = bool(args.fp16)
    return args


if __name__ == "__main__":
    a = parse_args()
    for k, v in vars(a).items():
        print(f"  {k}: {v}, type: {type(v)}")
    main(a)
