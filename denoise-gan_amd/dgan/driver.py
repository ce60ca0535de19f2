"""What the reference's four training drivers share around their train_step
(train_pix2pix.py:112-195, train_srgan.py:180-259, train_fsrgan.py:181-261,
train_autoencoder.py:169-241): output directories, the summary writer, the
tf.train.Checkpoint / CheckpointManager pair (max_to_keep=3, saved every 5th
epoch and at the end), --retrain restore, the epoch loop and its timing
print.

Differences from the reference, all needed for an exact resume:
  * the checkpoint also tracks the container's host counters (`epochs`,
    `iterations`) and the DataLoader continues from the restored epoch, so
    N epochs + resume + M epochs ends bit-identical to N + M epochs;
  * `model.epochs` is incremented before the epoch's checkpoint save;
  * data-parallel runs average the BN moving statistics across replicas
    (dgan.dist.sync_bn_stats) before a save, and only rank 0 writes files.
"""
import glob
import os
from time import time

import numpy as np
import torch

from . import summary as tf_summary
from .checkpoint import Checkpoint, CheckpointManager


class TrainState:
    """The container's host counters as a checkpointable object."""

    def __init__(self, model):
        self.model = model

    def state_dict(self):
        return {"epochs": np.array(self.model.epochs, np.int64), "iterations": np.array(self.model.iterations, np.int64)}

    def load_state_dict(self, d):
        if "epochs" in d:
            self.model.epochs = int(d["epochs"])
        if "iterations" in d:
            self.model.iterations = int(d["iterations"])


def is_chief():
    import torch.distributed as dist
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


def prepare(args):
    """Directories and the summary writer (train_pix2pix.py:117-142)."""
    for d in (os.path.join(args.model_dir, "checkpoints"), os.path.join(args.model_dir, "backups"), args.logdir):
        os.makedirs(d, exist_ok=True)
    traindirs = glob.glob(os.path.join(args.logdir, "train_*"))
    train_num = max([int(x.split("_")[-1]) for x in traindirs]) + 1 if traindirs else 1
    return tf_summary.create_file_writer(os.path.join(args.logdir, f"train_{train_num}"))


def make_checkpoint(model, args):
    ckpt = Checkpoint(gen_optimizer=model.gen_optimizer, disc_optimizer=model.disc_optimizer,
                      generator=model.generator, discriminator=model.discriminator, train_state=TrainState(model))
    return ckpt, CheckpointManager(ckpt, os.path.join(args.model_dir, "checkpoints"), max_to_keep=3)


def sync_before_save(model):
    if getattr(model, "grad_sync", None) is not None:
        from .dist import sync_bn_stats
        sync_bn_stats(model)


def run(args, model, ds, train, save_final=None):
    """The epoch loop of every driver: restore (--retrain), train epochs,
    checkpoint every 5th epoch, final save.  train(model, ds, args, writer)
    runs one epoch; save_final(model, timestamp) writes the exported weights."""
    from datetime import datetime
    writer = prepare(args)
    ckpt, manager = make_checkpoint(model, args)
    if bool(args.retrain) and manager.latest_checkpoint:
        ckpt.restore(manager.latest_checkpoint).expect_partial()
    if hasattr(ds, "set_epoch"):
        ds.set_epoch(model.epochs)
    print(f"Steps per epoch: {len(ds)}")
    timestamp = datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
    for epoch in range(args.epochs):
        t0 = time()
        train(model, ds, args, writer)
        torch.cuda.synchronize()
        t1 = time()
        model.epochs += 1
        if args.ckpt and epoch % 5 == 0:
            sync_before_save(model)
            if is_chief():
                manager.save()
        end = time()
        print(f"====== Finished epoch: {epoch + 1}, iterations: {model.iterations}, "
              f"train time: {t1 - t0:0.2f}, total time: {end - t0:0.2f} ======")
    if args.save_model:
        sync_before_save(model)
        if is_chief():
            manager.save()
            if save_final is not None:
                save_final(model, timestamp)
    return model
