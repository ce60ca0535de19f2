"""tf.train.Checkpoint / CheckpointManager stand-ins (train_pix2pix.py:156-164, :176-178).

A checkpoint is one .npz holding every tracked network's variables, BN moving
statistics and Adam slots (m, v, iterations; with mixed_float16 also the dynamic
loss scale: scale, good steps) under Keras-style names."""
import glob
import os
import re

import numpy as np
import torch


class Checkpoint:
    def __init__(self, **objects):
        self.objects = objects
        self.save_counter = 0

    def _collect(self):
        out = {}
        for key, obj in self.objects.items():
            arena = getattr(obj, "arena", None) or getattr(obj, "_arena", None)
            if hasattr(obj, "state_dict"):          # network
                for n, a in obj.state_dict().items():
                    out[f"{key}/{n}"] = a
            elif arena is not None:                   # optimizer bound to an arena
                out[f"{key}/m"] = arena.m.cpu().numpy()
                out[f"{key}/v"] = arena.v.cpu().numpy()
                out[f"{key}/iterations"] = arena.iterations.cpu().numpy()
                ls = getattr(obj, "_ls", None)
                if ls is not None:   # LossScaleOptimizer: current_loss_scale, good_steps (+ flag)
                    out[f"{key}/loss_scale"] = ls.cpu().numpy()
        return out

    def save(self, file_prefix):
        self.save_counter += 1
        path = f"{file_prefix}-{self.save_counter}.npz"
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        np.savez(path, **self._collect())
        return path

    def restore(self, path):
        if path is None:
            return self
        with np.load(path, allow_pickle=False) as z:
            data = {k: z[k] for k in z.files}
        for key, obj in self.objects.items():
            pre = f"{key}/"
            sub = {k[len(pre):]: v for k, v in data.items() if k.startswith(pre)}
            if hasattr(obj, "load_state_dict"):
                obj.load_state_dict(sub)
            else:
                arena = getattr(obj, "_arena", None)
                if arena is not None and "m" in sub:
                    arena.m.copy_(torch.as_tensor(sub["m"]))
                    arena.v.copy_(torch.as_tensor(sub["v"]))
                    arena.iterations.copy_(torch.as_tensor(sub["iterations"]))
                ls = getattr(obj, "_ls", None)
                if ls is not None and "loss_scale" in sub:
                    ls.copy_(torch.as_tensor(sub["loss_scale"]))
        m = re.search(r"-(\d+)\.npz$", path)
        if m:
            self.save_counter = int(m.group(1))
        return self

    def expect_partial(self):
        return self


class CheckpointManager:
    def __init__(self, checkpoint, directory, max_to_keep=3):
        self.checkpoint = checkpoint
        self.directory = directory
        self.max_to_keep = max_to_keep
        os.makedirs(directory, exist_ok=True)
        self.checkpoint.save_counter = max([self._num(p) for p in self._all()] + [0])

    @staticmethod
    def _num(p):
        m = re.search(r"-(\d+)\.npz$", p)
        return int(m.group(1)) if m else 0

    def _all(self):
        return sorted(glob.glob(os.path.join(self.directory, "ckpt-*.npz")), key=self._num)

    @property
    def latest_checkpoint(self):
        a = self._all()
        return a[-1] if a else None

    @property
    def checkpoints(self):
        return self._all()

    def save(self):
        path = self.checkpoint.save(os.path.join(self.directory, "ckpt"))
        for old in self._all()[:-self.max_to_keep]:
            os.remove(old)
        return path
