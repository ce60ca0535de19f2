"""SRGAN training driver — drop-in for the reference's train_srgan.py.

`train_step(model, x, y)` keeps the reference signature and its
7-tuple return (train_srgan.py:61-118); it runs the whole step (G/D
forwards, VGG content loss, losses, both gradients, Adam with
ExponentialDecay on G then D) as one launch sequence on libdgan
(dgan.sr_trainer.SRTrainer).  `train` / `main` follow the reference's loop
with the shared driver loop (dgan.driver), JSONL summaries and .npz weights.
"""
import os
from argparse import ArgumentParser

import numpy as np
import torch

from dataloader import DataLoader
from srgan import SRGAN
from dgan import driver
from dgan.models import to_device

LOSS_NAMES = ("gen_loss", "adv_loss", "mae_loss", "mse_loss", "content_loss", "disc_loss", "var_loss")


def train_step(model, x, y):
    """Single SRGAN step.  x: low-res batch, y: high-res batch (NHWC, [-1, 1]).
    Returns (gen_loss, adv_loss, mae_loss, mse_loss, content_loss, disc_loss,
    var_loss) as device scalars (train_srgan.py:118)."""
    x = to_device(x, model.device)
    y = to_device(y, model.device)
    loss = model.trainer(x.shape, y.shape).step(x, y)
    # loss = (gen_total, adv, mae, mse, content, disc, var)
    return tuple(loss[i] for i in range(7))


def train(model, dataset, args, writer):
    with writer.as_default():
        for x, y in dataset:
            losses = train_step(model, x, y)
            model.iterations += 1
            if model.iterations % args.save_iter == 0:
                vals = torch.stack(losses).cpu().numpy()
                for n, v in zip(LOSS_NAMES, vals):
                    writer.scalar(n, v, step=model.iterations)
                gen = model.generator(x, training=False)
                writer.image("Images/Generated", (255 * (gen.cpu().numpy() + 1) / 2).astype(np.uint8),
                             step=model.iterations)
                writer.flush()


def get_path(path):
    return os.path.realpath(os.path.expanduser(os.path.expandvars(path)))


def save_final(model, timestamp):
    name = model.model_name
    model.generator.save(os.path.join(model.model_dir, f"{name}.npz"))
    model.discriminator.save(os.path.join(model.model_dir, f"discriminator_{name}.npz"))
    model.generator.save(os.path.join(model.model_dir, "backups", f"{name}_{timestamp}.npz"))


def main(args):
    """The reference's main (dgan.driver.run: restore, epochs, checkpoints, exports)."""
    ds = DataLoader(args).dataset()
    model = SRGAN(args)
    model.model_dir, model.model_name = args.model_dir, args.model_name
    return driver.run(args, model, ds, train, save_final)


params = dict(
    model_name="srgan",
    image_dir=get_path("train/image_input/DIV2K_train_HR"),
    model_dir=get_path("./models"),
    logdir=get_path("./logs"),
    batch_size=1,
    epochs=1,
    crop_size=96,
    lr=1e-3,
    save_iter=200,
    retrain=0,
    save_model=1,
    ckpt=1,
    fp16=1,
    scale=4,
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
    args.model_name = args.model_name + f"_{args.scale}x_{args.jpeg_quality}q"
    if args.fp16:   # train_srgan.py:312-314: fp16 runs export under their own name
        args.model_name = args.model_name + "_fp16"
    return args


if __name__ == "__main__":
    a = parse_args()
    for k, v in vars(a).items():
        print(f"  {k}:".ljust(20) + f"{v!r}")
    main(a)
