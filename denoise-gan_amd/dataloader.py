"""DataLoader — drop-in for the reference's dataloader.py:9-229.

The host-side input pipeline of the training drivers.  It restates the
reference's tf.data pipeline on numpy + PIL (TensorFlow is not available):

  list_files(image_dir/*/*)          dataloader.py:27, :201   (shuffled order)
  load_image: decode to RGB float32 in [0, 1]; an image smaller than the crop
      in either dimension is resized to crop x crop (bilinear)     :31-59
  generate_image_pairs: (low, high) = (high, high)               :95-108
  stack_crop: one random crop x crop window for both             :79-93
  scale_image: low = resize(high, crop // scale, bicubic)        :110-125
      (tf.image.resize bicubic, antialias off = ResizeBicubic with
      half-pixel centres: Keys cubic a = -0.5, taps outside the image get
      weight 0 and the rest are renormalised, tap weights from a
      1024-entry table; restated in `resize_bicubic`)
  adjust_jpeg_quality(low, jpeg_quality): float -> uint8 (TF
      convert_image_dtype: floor(x * 255.5), saturated), JPEG encode at
      that quality (4:2:0), decode, / 255                         :127-140
  normalize: v * 2 - 1                                            :161-177
  cache -> shuffle(train_size) -> batch(drop_remainder=True)     :221
      (as in the reference, `cache()` follows the random crop, so every
      image keeps its first-epoch crop; batches are reshuffled each epoch)

The JPEG codec is PIL's libjpeg where the reference uses TF's; both are
libjpeg(-turbo) with the same quality / subsampling, but bit-identical
output is not claimed (parity of the training step is pinned on synthetic
pairs).

`args.synthetic = 1` replaces the files with seeded synthetic noisy/clean
pairs of the same contract (clean y = tanh(2 * bilinear-up(N(0,1) at 1/8
res)), noisy x = clip(y + N(0, 0.1^2), -1, 1)); that is what bench.py and
the tests train on.  Without it, an image_dir with no images is an error.
"""
import glob
import io
import os

import numpy as np


def get_path(path):
    return os.path.realpath(os.path.expanduser(os.path.expandvars(path)))


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


# ---------------------------------------------------------------------------
# TF resize restatements (half-pixel centres, no antialiasing)
# ---------------------------------------------------------------------------
_TABLE = 1024


def _keys_table(a=-0.5):
    """TF's bicubic coefficient table: for delta = i / 1024, the weights of the
    taps at distance 1 + delta, delta, 1 - delta, 2 - delta."""
    def w(t):
        t = np.abs(t)
        return np.where(t <= 1, ((a + 2) * t - (a + 3)) * t * t + 1,
                        np.where(t < 2, ((t - 5) * t + 8) * t * a - 4 * a, 0.0))
    d = np.arange(_TABLE + 1) / _TABLE
    return np.stack([w(1 + d), w(d), w(1 - d), w(2 - d)], axis=1)


_COEFFS = _keys_table()


def _bicubic_matrix(n_in, n_out):
    """[n_out, n_in] interpolation matrix of ResizeBicubic(half_pixel_centers=True)."""
    scale = n_in / n_out
    m = np.zeros((n_out, n_in), np.float64)
    for o in range(n_out):
        x = (o + 0.5) * scale - 0.5
        i = int(np.floor(x))
        off = int(np.rint((x - i) * _TABLE))
        wts = _COEFFS[off].copy()
        idx = np.array([i - 1, i, i + 1, i + 2])
        inside = (idx >= 0) & (idx < n_in)
        wts = np.where(inside, wts, 0.0)
        s = wts.sum()
        if abs(s) > 0:
            wts = wts / s
        for k in range(4):
            if inside[k]:
                m[o, idx[k]] += wts[k]
    return m


def resize_bicubic(img, h, w):
    """tf.image.resize(img, [h, w], method='bicubic') for an HWC float image."""
    my = _bicubic_matrix(img.shape[0], h)
    mx = _bicubic_matrix(img.shape[1], w)
    out = np.einsum("oh,hwc->owc", my, img.astype(np.float64))
    out = np.einsum("pw,owc->opc", mx, out)
    return out.astype(np.float32)


def _bilinear_matrix(n_in, n_out):
    scale = n_in / n_out
    m = np.zeros((n_out, n_in), np.float64)
    for o in range(n_out):
        x = max((o + 0.5) * scale - 0.5, 0.0)
        i0 = min(int(np.floor(x)), n_in - 1)
        i1 = min(i0 + 1, n_in - 1)
        f = x - i0
        m[o, i0] += 1 - f
        m[o, i1] += f
    return m


def resize_bilinear(img, h, w):
    """tf.image.resize(img, [h, w]) (bilinear, half-pixel centres) for an HWC float image."""
    out = np.einsum("oh,hwc->owc", _bilinear_matrix(img.shape[0], h), img.astype(np.float64))
    return np.einsum("pw,owc->opc", _bilinear_matrix(img.shape[1], w), out).astype(np.float32)


def to_uint8(img):
    """tf.image.convert_image_dtype(float -> uint8, saturate=True)."""
    return np.clip(np.floor(img.astype(np.float64) * 255.5), 0, 255).astype(np.uint8)


def jpeg_roundtrip(img, quality):
    """tf.image.adjust_jpeg_quality: uint8 conversion, JPEG encode / decode, back to [0, 1]."""
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(to_uint8(img), "RGB").save(buf, format="JPEG", quality=int(quality), subsampling=2)
    buf.seek(0)
    return np.asarray(Image.open(buf).convert("RGB"), np.float32) / 255.0


# ---------------------------------------------------------------------------
class DataLoader(object):
    """Data loader of the training drivers (dataloader.py:9-229)."""

    def __init__(self, args):
        self.image_dir = getattr(args, "image_dir", "")
        self.crop_size = int(args.crop_size)
        self.scale = int(getattr(args, "scale", 1))
        self.jpeg_quality = int(getattr(args, "jpeg_quality", 50))
        self.batch_size = int(args.batch_size)
        self.seed = int(getattr(args, "seed", 0))
        self.synthetic = bool(int(getattr(args, "synthetic", 0)))
        self._epoch = 0
        self._cache = None
        if self.synthetic:
            self.image_paths = []
            self.steps = int(getattr(args, "steps_per_epoch", 0) or 8)
            self.train_size = self.steps * self.batch_size
        else:
            self.image_paths = sorted(p for p in glob.glob(os.path.join(self.image_dir, "*/*")) if os.path.isfile(p))
            self.train_size = len(self.image_paths)
            if self.train_size == 0:
                raise FileNotFoundError(
                    f"no images under {os.path.join(self.image_dir, '*/*')} (dataloader.py:27 layout); "
                    "pass --synthetic 1 to train on seeded synthetic pairs")
            self.steps = self.train_size // self.batch_size

    def set_epoch(self, epoch):
        """Position the epoch counter (a resumed run continues the batch order)."""
        self._epoch = int(epoch)

    # --- per-image maps (dataloader.py:31-177) -----------------------------
    def load_image(self, image_path):
        from PIL import Image
        with Image.open(image_path) as im:
            image = np.asarray(im.convert("RGB"), np.float32) / 255.0
        if image.shape[0] < self.crop_size or image.shape[1] < self.crop_size:
            image = resize_bilinear(image, self.crop_size, self.crop_size)
        return image

    def generate_image_pairs(self, high_res):
        return high_res, high_res

    def stack_crop(self, image_input, image_target, rng):
        c = self.crop_size
        oy = int(rng.integers(0, image_target.shape[0] - c + 1))
        ox = int(rng.integers(0, image_target.shape[1] - c + 1))
        return image_input[oy:oy + c, ox:ox + c], image_target[oy:oy + c, ox:ox + c]

    def scale_image(self, low_res, high_res):
        s = self.crop_size // self.scale
        return resize_bicubic(high_res, s, s), high_res

    def adjust_jpeg_quality(self, low_res, high_res):
        return jpeg_roundtrip(low_res, self.jpeg_quality), high_res

    def normalize(self, image_input, image_target):
        return image_input * 2 - 1, image_target * 2 - 1

    # --- dataset -----------------------------------------------------------
    def _build_cache(self):
        rng = np.random.Generator(np.random.PCG64(self.seed))
        order = rng.permutation(self.train_size)        # list_files shuffles
        pairs = []
        for i in order:
            hi = self.load_image(self.image_paths[i])
            lo, hi = self.generate_image_pairs(hi)
            lo, hi = self.stack_crop(lo, hi, rng)
            lo, hi = self.scale_image(lo, hi)
            lo, hi = self.adjust_jpeg_quality(lo, hi)
            pairs.append(self.normalize(lo, hi))
        self._cache = pairs

    def dataset(self):
        return self

    def __iter__(self):
        epoch = self._epoch
        self._epoch += 1
        if self.synthetic:
            base = self.seed * 100003 + epoch * 1009
            for i in range(self.steps):
                x, y = synthetic_pair(self.batch_size, self.crop_size, seed=base + i)
                if self.scale > 1:
                    x = np.ascontiguousarray(x[:, ::self.scale, ::self.scale, :])
                yield x, y
            return
        if self._cache is None:
            self._build_cache()
        perm = np.random.Generator(np.random.PCG64([self.seed, epoch])).permutation(self.train_size)
        B = self.batch_size
        for b in range(self.steps):
            idx = perm[b * B:(b + 1) * B]
            yield (np.stack([self._cache[i][0] for i in idx]).astype(np.float32),
                   np.stack([self._cache[i][1] for i in idx]).astype(np.float32))

    def __len__(self):
        return self.steps
