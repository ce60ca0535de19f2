"""DataLoader semantics (dataloader.py:9-229 restated on numpy + PIL): TF
resize known answers, the crop / bicubic / JPEG / [-1, 1] pipeline over a
directory of images, epoch order and drop_remainder."""
import os

import numpy as np
import pytest

import dataloader as DL


class Args:
    def __init__(self, **kw):
        self.crop_size = 32
        self.scale = 2
        self.jpeg_quality = 90
        self.batch_size = 2
        self.seed = 3
        self.__dict__.update(kw)


def test_bicubic_known_answers():
    rng = np.random.default_rng(0)
    img = rng.uniform(size=(12, 10, 3)).astype(np.float32)
    # same size: every output pixel samples an input centre exactly (weights 0, 1, 0, 0)
    assert np.allclose(DL.resize_bicubic(img, 12, 10), img, atol=1e-6)
    # constants stay constant (weights renormalised at the borders)
    c = np.full((9, 7, 3), 0.25, np.float32)
    assert np.allclose(DL.resize_bicubic(c, 4, 3), 0.25, atol=1e-6)
    # 2x down, half-pixel centres: output o samples x = 2o + 0.5 -> Keys(-0.5) weights
    # (-1/16, 9/16, 9/16, -1/16) on rows 2o-1 .. 2o+2; row 0 drops the outside tap and renormalises
    m = DL._bicubic_matrix(8, 4)
    assert np.allclose(m[1, 1:5], [-0.0625, 0.5625, 0.5625, -0.0625])
    assert np.allclose(m[0, :3], np.array([0.5625, 0.5625, -0.0625]) / 1.0625)
    assert np.allclose(m.sum(1), 1.0)


def test_bilinear_upscale_and_uint8():
    img = np.arange(4, dtype=np.float32).reshape(2, 2, 1).repeat(3, -1) / 3
    up = DL.resize_bilinear(img, 4, 4)
    # half-pixel centres: out 0 -> x = -0.25 clamps to 0; out 1 -> x = 0.25
    assert np.isclose(up[0, 0, 0], 0.0) and np.isclose(up[1, 0, 0], 0.25 * 2 / 3)
    assert DL.to_uint8(np.array([0.0, 0.5, 1.0, 1.2]))[1] == 127  # floor(0.5 * 255.5)
    assert DL.to_uint8(np.array([0.0, 0.5, 1.0, 1.2]))[3] == 255


def _image_dir(tmp_path, n=5):
    from PIL import Image
    rng = np.random.default_rng(1)
    root = tmp_path / "DIV2K" / "sub"
    root.mkdir(parents=True)
    sizes = [(48, 40), (40, 56), (64, 64), (20, 24), (50, 50)][:n]
    imgs = {}
    for i, (h, w) in enumerate(sizes):
        yy, xx = np.mgrid[0:h, 0:w]
        a = np.stack([np.sin(yy / 5.0 + i), np.cos(xx / 7.0), np.sin((xx + yy) / 9.0)], -1)
        a = ((a + 1) * 127.5 + rng.normal(0, 4, a.shape)).clip(0, 255).astype(np.uint8)
        p = root / f"img{i}.png"
        Image.fromarray(a).save(p)
        imgs[str(p)] = a
    return str(tmp_path / "DIV2K"), imgs


def test_pipeline_over_image_files(tmp_path):
    image_dir, imgs = _image_dir(tmp_path)
    ld = DL.DataLoader(Args(image_dir=image_dir))
    assert ld.train_size == 5 and len(ld) == 2          # drop_remainder
    batches = list(ld.dataset())
    assert len(batches) == 2
    for x, y in batches:
        assert x.shape == (2, 16, 16, 3) and y.shape == (2, 32, 32, 3)
        assert x.dtype == np.float32 and y.dtype == np.float32
        assert x.min() >= -1 and x.max() <= 1 and y.min() >= -1 and y.max() <= 1
        for k in range(2):
            # x = JPEG(bicubic(y)) at quality 90: close to the bicubic downscale of y
            ref = DL.resize_bicubic((y[k] + 1) / 2, 16, 16)
            mse = np.mean(((x[k] + 1) / 2 - ref) ** 2)
            assert 10 * np.log10(1 / mse) > 28
    # every target is a crop of one image (or of the 20x24 image resized up to 32x32)
    srcs = [a.astype(np.float32) / 255 for a in imgs.values()]
    y0 = (batches[0][1][0] + 1) / 2
    found = False
    for a in srcs:
        if a.shape[0] < 32 or a.shape[1] < 32:
            a = DL.resize_bilinear(a, 32, 32)
        for oy in range(a.shape[0] - 31):
            for ox in range(a.shape[1] - 31):
                if np.allclose(a[oy:oy + 32, ox:ox + 32], y0, atol=1e-6):
                    found = True
    assert found
    # cache: crops fixed after the first epoch, order reshuffled per epoch, reproducible
    e1 = list(ld.dataset())
    all0 = sorted(map(lambda t: t.tobytes(), np.concatenate([b[1] for b in batches])))
    all1 = sorted(map(lambda t: t.tobytes(), np.concatenate([b[1] for b in e1])))
    assert len(set(all0) & set(all1)) >= 3
    ld2 = DL.DataLoader(Args(image_dir=image_dir))
    ld2.set_epoch(1)
    e1b = list(ld2.dataset())
    for (a, b), (c, d) in zip(e1, e1b):
        assert np.array_equal(a, c) and np.array_equal(b, d)


def test_missing_images_fail_loudly_and_synthetic_flag(tmp_path):
    with pytest.raises(FileNotFoundError):
        DL.DataLoader(Args(image_dir=str(tmp_path)))
    ld = DL.DataLoader(Args(image_dir=str(tmp_path), synthetic=1, steps_per_epoch=3, scale=4))
    b = list(ld.dataset())
    assert len(b) == 3 and b[0][0].shape == (2, 8, 8, 3) and b[0][1].shape == (2, 32, 32, 3)
