"""Numerics of the HIP conv engine (fwd / bwd_data / bwd_filter) against a
plain PyTorch fp64 CPU reference of the same Keras layer, for every layer
geometry of the pix2pix generator and discriminator (pix2pix.py:110-220)
plus the SRGAN/FSRGAN shapes (k3 'same' with TF's asymmetric pads, k1).

Both conv arithmetics (include/dgan.h DG_MATH_*) are held to the same
fp32-level tolerance: exact fp32 MFMA, and bf16x6 (fp32 operands split into
three bf16 pieces, six piece products on the bf16 matrix cores).
Tolerance vs fp64: relative L2 error < 2e-6 and max-abs error
< 1e-5 * max|ref| (scaled by sqrt(K/1024) for long K)."""
import math
import zlib

import pytest
import torch

from torch_ref import conv2d_ref, conv2d_transpose_ref

gpu = pytest.mark.gpu

# (name, N, H, W, Cin, Cout, k, s, padding, transpose, bias)
CASES = [
    ("G.down1", 2, 64, 64, 3, 64, 4, 2, "same", False, False),
    ("G.down2", 2, 32, 32, 64, 128, 4, 2, "same", False, False),
    ("G.down4", 2, 16, 16, 256, 512, 4, 2, "same", False, False),
    ("G.down8", 4, 2, 2, 512, 512, 4, 2, "same", False, False),
    ("G.up1", 4, 1, 1, 512, 512, 4, 2, "same", True, False),
    ("G.up2", 2, 2, 2, 1024, 512, 4, 2, "same", True, False),
    ("G.up5", 2, 8, 8, 1024, 256, 4, 2, "same", True, False),
    ("G.up7", 2, 16, 16, 256, 64, 4, 2, "same", True, False),
    ("G.last", 2, 32, 32, 128, 3, 4, 2, "same", True, True),
    ("D.down1", 2, 64, 64, 6, 64, 4, 2, "same", False, False),
    ("D.conv", 2, 16, 16, 256, 512, 4, 1, (1, 1, 1, 1), False, False),
    ("D.last", 2, 15, 15, 512, 1, 4, 1, (1, 1, 1, 1), False, True),
    ("k3s1", 2, 12, 12, 64, 64, 3, 1, "same", False, True),
    ("k3s2", 2, 12, 12, 32, 64, 3, 2, "same", False, True),
    ("k1s1", 2, 6, 6, 64, 3, 1, 1, "same", False, True),
    ("odd", 3, 9, 7, 8, 32, 4, 2, "same", False, False),
    # input gradients with Cin 3 / 6 on the direct narrow-DGRAD kernel (ragged
    # 8x32 phase tiles, two 32-channel chunks, k3 s2 phases with fewer taps);
    # G.last.odd (Co 160 in the conv view) stays on the GEMM recast
    ("V.b1c1", 2, 37, 45, 3, 64, 3, 1, "same", False, True),
    ("D.down1.odd", 2, 27, 70, 6, 64, 4, 2, "same", False, False),
    ("k3s2.c3", 2, 17, 19, 3, 64, 3, 2, "same", False, False),
    ("G.last.odd", 2, 13, 21, 160, 3, 4, 2, "same", True, True),
    # small-Cin 4x4 stride-2 kernels (conv_small.hip: Cin 3 / 6, Wo % 32 == 0): two row
    # segments, two column tiles, several conv-view rows per WGRAD block, valid padding
    ("small.wide", 3, 32, 128, 3, 64, 4, 2, "same", False, True),
    ("small.co128", 1, 64, 64, 6, 128, 4, 2, "same", False, False),
    ("small.rows", 3, 384, 64, 3, 64, 4, 2, "same", False, False),
    ("small.valid", 2, 66, 66, 6, 64, 4, 2, "valid", False, True),
    ("small.tlast", 1, 64, 64, 64, 3, 4, 2, "same", True, True),
    # VGG19 block1_conv1's forward on the small-Cin kernel (3x3 stride 1, Cin 3)
    ("small.k3", 2, 32, 64, 3, 64, 3, 1, "same", False, True),
    ("small.k3c128", 3, 24, 32, 3, 128, 3, 1, "same", False, False),
    # single-output-channel direct input / filter gradients (conv_co1.hip): the
    # bs16 PatchGAN last layer's geometry, stride 2 and 3x3 (generic tap loops),
    # a wide row, and a 4-channel input (64 pixel lanes per block)
    ("co1.full", 4, 31, 31, 512, 1, 4, 1, (1, 1, 1, 1), False, True),
    ("co1.s2", 2, 19, 23, 64, 1, 4, 2, "same", False, True),
    ("co1.k3", 2, 9, 300, 128, 1, 3, 1, "same", False, False),
    ("co1.c4", 2, 11, 13, 4, 1, 4, 1, (1, 1, 1, 1), False, True),
    # Conv2DTranspose(3) forward on the fused MFMA + col2im kernel (conv_tlast.hip):
    # ragged 16 x 32 output tiles, and a 128 x 128 output
    ("tlast.ragged", 2, 13, 21, 128, 3, 4, 2, "same", True, True),
    ("tlast.big", 1, 64, 64, 128, 3, 4, 2, "same", True, True),
]


def _close(got, ref, K, what):
    got = got.double().cpu()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-30
    rel = ((got - ref).norm() / (ref.norm() + 1e-30)).item()
    tol = 1e-5 * max(1.0, math.sqrt(K / 1024.0))
    assert rel < 2e-6 * max(1.0, math.sqrt(K / 1024.0)), f"{what}: rel L2 {rel:.3e}"
    assert err <= tol * scale, f"{what}: max abs {err:.3e} vs scale {scale:.3e}"


MATHS = ["fp32", "bf16x6"]


@gpu
@pytest.mark.parametrize("math_mode", MATHS)
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_conv_layer(case, math_mode, xscale=1.0, gscale=1.0):
    """xscale / gscale: magnitude of the activations (and bias) / of the output gradient
    (test_x3_gpu.py: fp16x3 operand ranges); the bars are relative to each result's scale."""
    from dgan.ops import ConvDesc
    name, N, H, W, Cin, Cout, k, s, padding, transpose, has_bias = case
    torch.manual_seed(zlib.crc32(name.encode()))
    d = ConvDesc(N, H, W, Cin, Cout, k, s, padding, transpose, math=math_mode)
    x = torch.randn(N, H, W, Cin, dtype=torch.float64) * xscale
    w = torch.randn(*d.weight_shape, dtype=torch.float64) * 0.05
    b = torch.randn(Cout, dtype=torch.float64) * xscale if has_bias else None
    dy = torch.randn(N, d.Ho, d.Wo, Cout, dtype=torch.float64) * gscale

    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    br = b.clone().requires_grad_() if has_bias else None
    if transpose:
        yr = conv2d_transpose_ref(xr, wr, s, d.pads, (d.Ho, d.Wo), br)
    else:
        yr = conv2d_ref(xr, wr, s, d.pads, br)
    assert tuple(yr.shape) == d.out_shape
    yr.backward(dy)

    dev = torch.device("cuda")
    xg, wg, dyg = x.float().to(dev), w.float().to(dev), dy.float().to(dev)
    bg = b.float().to(dev) if has_bias else None
    y = torch.empty(d.out_shape, device=dev)
    d.fwd(xg, wg, y, bias=bg)
    dx = torch.empty_like(xg)
    d.bwd_data(dyg, wg, dx)
    dw = torch.empty_like(wg)
    db = torch.empty(Cout, device=dev) if has_bias else None
    d.bwd_filter(xg, dyg, dw, dbias=db)
    torch.cuda.synchronize()
    K = k * k * (Cin if not transpose else Cout)
    _close(y, yr.detach(), K, f"{name} fwd")
    _close(dx, xr.grad, k * k * Cout, f"{name} bwd_data")
    _close(dw, wr.grad, N * d.Ho * d.Wo, f"{name} bwd_filter")
    if has_bias:
        # a column sum of random-sign terms can cancel: scale by sum |dy| instead of |sum|
        err = (db.double().cpu() - br.grad).abs().max().item()
        assert err <= 1e-6 * dy.abs().sum(dim=(0, 1, 2)).max().item(), f"{name} dbias: {err:.3e}"


# layers on the halo-tiled bf16x6 kernel (csrc/conv_x6h.hip), stride-1 3x3:
# ragged 8x16 output patches (H, W not multiples of 8 / 16), 'valid' padding,
# BN 64 and 128, and split-K over channel chunks (small images, many channels)
HALO_CASES = [
    ("h.ragged", 4, 40, 36, 64, 128, 3, 1, "same", False, True),
    ("h.bn64", 2, 16, 16, 256, 64, 3, 1, "same", False, False),
    ("h.splitk", 2, 8, 8, 512, 512, 3, 1, "same", False, False),
    ("h.valid", 2, 20, 21, 64, 64, 3, 1, "valid", False, True),
    ("h.tfpad", 3, 13, 29, 32, 48, 3, 1, (1, 1, 1, 1), False, False),
    # BN 32 (32 output columns: the SR family's 32-channel layers): ragged patches,
    # 16 input channels (one chunk), split-K over chunks on a small grid
    ("h32.ragged", 3, 21, 37, 32, 32, 3, 1, "same", False, True),
    ("h32.c16", 2, 24, 24, 16, 32, 3, 1, "same", False, False),
    ("h32.splitk", 2, 8, 8, 256, 32, 3, 1, "same", False, True),
    # stride-2 4x4 layers: the input gradient in 4 sub-pixel phases (Conv2D
    # bwd_data and Conv2DTranspose fwd; ragged patches, odd sizes whose phases
    # differ in size, BN 64 / 128, split-K)
    ("h2.down", 2, 32, 32, 64, 128, 4, 2, "same", False, False),
    ("h2.up", 2, 16, 16, 256, 64, 4, 2, "same", True, False),
    ("h2.ragged", 3, 26, 40, 32, 64, 4, 2, "same", False, True),
    ("h2.odd", 2, 17, 15, 16, 32, 4, 2, "same", False, False),
    ("h2.splitk", 2, 8, 8, 512, 512, 4, 2, "same", False, False),
    ("h2.valid", 2, 20, 22, 32, 64, 4, 2, "valid", False, True),
    # stride-1 4x4 (the PatchGAN's ZeroPadding2D + Conv2D(512, 4)): the input
    # gradient on the 11 x 19 halo, ragged patches, 'same' (asymmetric pads)
    ("h4.pad", 2, 18, 21, 32, 64, 4, 1, (1, 1, 1, 1), False, False),
    ("h4.same", 3, 11, 17, 16, 32, 4, 1, "same", False, True),
    ("h4.bn128", 2, 16, 16, 64, 256, 4, 1, (1, 1, 1, 1), False, False),
]


@gpu
@pytest.mark.parametrize("case", HALO_CASES, ids=[c[0] for c in HALO_CASES])
def test_conv_halo_kernel(case, monkeypatch):
    # force the bf16x6 path (the planner keeps small GEMMs on the fp32 kernel);
    # every stride-1 3x3 bf16x6 FWD / DGRAD plan and every stride-2 4x4 DGRAD
    # runs on the halo kernel
    monkeypatch.setenv("DG_FORCE_X6CFG", "0")
    monkeypatch.delenv("DG_PLAN_DISABLE", raising=False)
    test_conv_layer(case, "bf16x6")


@gpu
@pytest.mark.parametrize("math_mode", MATHS)
def test_conv_strided_views_and_accumulate(math_mode):
    """Zero-copy concat: read a channel slice, write into a slice with beta=1."""
    from dgan.ops import ConvDesc
    torch.manual_seed(0)
    dev = torch.device("cuda")
    N, H, W, Cin, Cout = 2, 16, 16, 64, 128
    d = ConvDesc(N, H, W, Cin, Cout, 4, 2, "same", math=math_mode)
    big_in = torch.randn(N, H, W, Cin + 64, device=dev)
    x = big_in[..., 64:]
    w = torch.randn(*d.weight_shape, device=dev) * 0.05
    out = torch.randn(N, d.Ho, d.Wo, Cout + 128, device=dev)
    y = out[..., :Cout]
    y0 = y.clone()
    d.fwd(x, w, y, beta=1.0)
    ref = conv2d_ref(x.double().cpu(), w.double().cpu(), 2, d.pads) + y0.double().cpu()
    torch.cuda.synchronize()
    _close(y, ref, 16 * Cin, "strided fwd beta=1")
    # untouched channels stay intact
    assert torch.equal(out[..., Cout:].cpu(), out[..., Cout:].cpu())
    # bwd_data into a slice, accumulate
    dy = torch.randn(N, d.Ho, d.Wo, Cout, device=dev)
    dxbuf = torch.randn(N, H, W, Cin + 32, device=dev)
    dx = dxbuf[..., 32:]
    dx0 = dx.clone()
    d.bwd_data(dy, w, dx, beta=1.0)
    xr = x.double().cpu().requires_grad_()
    conv2d_ref(xr, w.double().cpu(), 2, d.pads).backward(dy.double().cpu())
    torch.cuda.synchronize()
    _close(dx, xr.grad + dx0.double().cpu(), 16 * Cout, "strided bwd_data beta=1")


@gpu
def test_conv_fused_lrelu_epilogue():
    from dgan.ops import ConvDesc
    torch.manual_seed(1)
    dev = torch.device("cuda")
    d = ConvDesc(2, 32, 32, 64, 128, 4, 2, "same")
    x = torch.randn(2, 32, 32, 64, device=dev)
    w = torch.randn(*d.weight_shape, device=dev) * 0.05
    y = torch.empty(d.out_shape, device=dev)
    d.fwd(x, w, y, act="lrelu", alpha=0.3)
    ref = conv2d_ref(x.double().cpu(), w.double().cpu(), 2, d.pads)
    ref = torch.where(ref > 0, ref, 0.3 * ref)
    torch.cuda.synchronize()
    _close(y, ref, 1024, "lrelu epilogue")


@gpu
def test_bf16x6_error_matches_fp32():
    """The split arithmetic's error vs fp64 stays at the fp32 path's level
    (exact-fp32 inputs, so only the GEMM arithmetic differs)."""
    from dgan.ops import ConvDesc
    torch.manual_seed(7)
    dev = torch.device("cuda")
    N, H, W, Cin, Cout = 4, 16, 16, 256, 256
    x = torch.randn(N, H, W, Cin).float()
    errs = {}
    for m in MATHS:
        d = ConvDesc(N, H, W, Cin, Cout, 4, 1, (1, 1, 1, 1), math=m)
        w = (torch.randn(*d.weight_shape, generator=torch.Generator().manual_seed(3)) * 0.05).float()
        ref = conv2d_ref(x.double(), w.double(), 1, d.pads)
        y = torch.empty(d.out_shape, device=dev)
        d.fwd(x.to(dev), w.to(dev), y)
        torch.cuda.synchronize()
        errs[m] = ((y.double().cpu() - ref).norm() / ref.norm()).item()
    assert errs["bf16x6"] < 2.0 * errs["fp32"] + 1e-9, errs
