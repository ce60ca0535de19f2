"""DataLoader stand-in (reference: dataloader.py:9-229).

The reference's tf.data pipeline (DIV2K files -> random crop -> bicubic down
-> JPEG degradation -> [-1, 1]) is out of scope for the hot path (SURVEY.md
§2 row 9); what the training step consumes is its output contract: batched
NHWC float32 pairs (x noisy, y clean) in [-1, 1] with drop_remainder=True
(dataloader.py:161-177, :221).  This loader produces seeded synthetic pairs
of that contract: clean y = tanh(2 * bilinear-up(N(0,1) at 1/8 res)), noisy
x = clip(y + N(0, 0.1^2), -1, 1) — a stand-in for JPEG degradation.
"""
import numpy as np


def synthetic_pair(batch, size, seed=0):
    rng = np.random.Generator(np.random.PCG64(seed))
    lo = max(1, size // 8)
    z = rng.standard_normal((batch, lo + 1, lo + 1, 3))
    t = np.linspace(0.0, lo, size)
    i0 = np.minimum(np.floor(t).astype(int), lo - 1)
    fr = t - i0
    zr = z[:, i0, :, :] * (1 - fr)[None, :, None, None] + z[:, i0 + 1, :, :] * fr[None, :, None, None]
    zc = zr[:, :, i0, :] * (1 - fr)[None, None, :, None] + zr[:, :, i0 + 1, :] * fr[None, None, :, None]
    y = np.tanh(2.0 * zc)
    x = np.clip(y + 0.1 * rng.standard_normal(y.shape), -1.0, 1.0)
    return np.ascontiguousarray(x, dtype=np.float32), np.ascontiguousarray(y, dtype=np.float32)


class DataLoader(object):
    def __init__(self, args):
        self.batch_size = int(args.batch_size)
        self.crop_size = int(args.crop_size)
        self.scale = int(getattr(args, "scale", 1))
        self.jpeg_quality = getattr(args, "jpeg_quality", 50)
        self.steps = int(getattr(args, "steps_per_epoch", 0) or 8)
        self.seed = int(getattr(args, "seed", 0))
        self._epoch = 0

    def dataset(self):
        return self

    def __iter__(self):
        base = self.seed * 100003 + self._epoch * 1009
        self._epoch += 1
        for i in range(self.steps):
            x, y = synthetic_pair(self.batch_size, self.crop_size, seed=base + i)
            if self.scale > 1:
                x = x[:, ::self.scale, ::self.scale, :]
            yield x, y

    def __len__(self):
        return self.steps
