"""The fp16x3 conv math (include/dgan.h DG_MATH_F16X3): three fp16 piece products of
pre-scaled operands (s x = h + l, h.h' + l.h' + h.l') -- the frozen VGG19's 3x3 stride-1
layers on the halo kernel (conv_x6h.hip NI 4; keras VGG19 blocks 1-5 after block1_conv1,
as built by pix2pix.py:53-67 / srgan.py:70-76) and the pix2pix G / D layers on the
implicit-GEMM kernel (conv_x6.hip NI 4; pix2pix.py:110-142, :194-220).

  * the layer against a torch fp64 reference at the conv engine's fp32 bar
    (test_conv_gpu.py _close: relative L2 < 2e-6, max-abs < 1e-5 of scale),
    forward, input and filter gradient (gradients scaled from their measured max);
  * the fp16x3 planes a producer writes beside its output (conv epilogue,
    fused pool epilogue, unfused max pool) are the bytes the layer's own split
    pass writes, so a fed forward is bit-identical to an unfed one;
  * the input gradient masked by the sign of the fp16x3 hi plane equals the
    one masked by the fp32 activation;
  * a mixed 2-layer chain (fused pool) ends bit-identical whether planes are
    fed or split."""
import pytest
import torch

from dgan import ops
from test_conv_gpu import _close, test_conv_layer

gpu = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _force_x3(monkeypatch):
    """Every fp16x3-eligible op on fp16x3, also where the planner would keep a small GEMM on the
    fp32 tiles (csrc/conv.hip make_plan): these cases exercise the kernels at small sizes."""
    monkeypatch.setenv("DG_FORCE_X3", "1")

# (name, N, H, W, Cin, Cout, k, s, padding, transpose, bias): VGG19-like layers on
# the fp16x3 halo kernel -- BN 64 / 128, ragged 8x16 patches, split-K over the
# 32-channel chunks (small image, many channels), 'valid' padding, Cout 48 (BN 64 tile
# with a ragged column block)
X3_CASES = [
    ("x3.b2", 2, 32, 32, 64, 128, 3, 1, "same", False, True),
    ("x3.bn64", 2, 16, 16, 128, 64, 3, 1, "same", False, False),
    ("x3.ragged", 3, 21, 37, 64, 128, 3, 1, "same", False, True),
    ("x3.splitk", 2, 8, 8, 512, 512, 3, 1, "same", False, True),
    ("x3.valid", 2, 20, 22, 32, 64, 3, 1, "valid", False, False),
    ("x3.c48", 2, 16, 24, 96, 48, 3, 1, "same", False, True),
    # the pix2pix G / D layers on the implicit-GEMM kernel (conv_x6.hip NI 4): 4x4 stride 2
    # down / up (the input gradient's 4 sub-pixel phases, ConvT forward), ragged and odd
    # sizes, the deep U-Net shapes (tiny M, split-K over 8192-16384 k), the PatchGAN's
    # stride-1 4x4
    ("x3.down", 2, 32, 32, 64, 128, 4, 2, "same", False, False),
    ("x3.up", 2, 16, 16, 256, 64, 4, 2, "same", True, False),
    ("x3.down.ragged", 3, 26, 40, 32, 64, 4, 2, "same", False, True),
    ("x3.up.odd", 2, 9, 7, 64, 32, 4, 2, "same", True, True),
    ("x3.deep", 4, 4, 4, 512, 512, 4, 2, "same", False, False),
    ("x3.deep.up", 4, 2, 2, 1024, 512, 4, 2, "same", True, False),
    ("x3.patch", 2, 18, 21, 64, 128, 4, 1, (1, 1, 1, 1), False, False),
    # the PatchGAN's stride-1 4x4 on the fp16x3 halo kernel (KT 4, forward and input gradient):
    # 'valid' on a zero-padded map as pix2pix.py:205-208 builds it, 8 channel chunks, ragged
    # patches, Cout 96 (a ragged BN 64 column block)
    ("x3.patch.valid", 2, 34, 27, 256, 96, 4, 1, "valid", False, True),
]


def _rand(shape, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).cuda()


@gpu
@pytest.mark.parametrize("case", X3_CASES, ids=[c[0] for c in X3_CASES])
def test_x3_layer_matches_fp64(case, monkeypatch):
    monkeypatch.delenv("DG_PLAN_DISABLE", raising=False)
    name, N, H, W, Cin, Cout, k, s, padding, transpose, bias = case
    d = ops.ConvDesc(N, H, W, Cin, Cout, k, s, padding, transpose, math="f16x3")
    assert d.plane_format(ops.TENSOR_X) == ops.PLANES_F16X3, f"{name}: forward not planned on fp16x3"
    test_conv_layer(case, "f16x3")


# operand magnitudes far from the unit-scale cases above: activations of
# 1e-3 and 1e3, output gradients of 1e-8 and 1e4 -- on the 3x3 halo kernel (forward / input
# gradient) and the implicit-GEMM kernel (4x4 stride-2 conv and ConvT, filter gradients
# included), each against fp64 at the same relative bar as the unit-scale cases
X3_SCALE_CASES = [(c, xs, gs) for c in (X3_CASES[0], X3_CASES[6], X3_CASES[7])
                  for xs, gs in ((1e-3, 1.0), (1e3, 1.0), (1.0, 1e-8), (1.0, 1e4), (1e-3, 1e-8))]


@gpu
@pytest.mark.parametrize("case,xs,gs", X3_SCALE_CASES,
                         ids=[f"{c[0]}-x{xs:g}-g{gs:g}" for c, xs, gs in X3_SCALE_CASES])
def test_x3_layer_at_operand_scales(case, xs, gs, monkeypatch):
    monkeypatch.delenv("DG_PLAN_DISABLE", raising=False)
    test_conv_layer(case, "f16x3", xscale=xs, gscale=gs)


# persistent halo blocks (conv_x6h.hip PERS: a block runs p.ptiles patches back to back, the
# next patch's halo and weights fetched under the current one's MFMAs): forced to 3 and 5
# patches per block on the halo cases -- patch counts that do not divide the grid, ragged
# edge patches, Cout 48, the 4x4 stride-2 input-gradient / ConvT-forward phases -- at the
# same fp64 bar (the planner applies it only to grids of >= 1024 patches, beyond these sizes)
X3_PERS_CASES = [(c, pt) for c in (X3_CASES[0], X3_CASES[1], X3_CASES[2], X3_CASES[4], X3_CASES[5],
                                   X3_CASES[6], X3_CASES[7], X3_CASES[8], X3_CASES[12], X3_CASES[13])
                 for pt in (3, 5)]


@gpu
@pytest.mark.parametrize("case,pt", X3_PERS_CASES, ids=[f"{c[0]}-pt{pt}" for c, pt in X3_PERS_CASES])
def test_x3_persistent_blocks_match_fp64(case, pt, monkeypatch):
    monkeypatch.delenv("DG_PLAN_DISABLE", raising=False)
    monkeypatch.setenv("DG_X3H_PTILES", str(pt))
    test_conv_layer(case, "f16x3")


# the 16 x 16 patch on 8 waves (conv_x6h.hip PH 16, round 6): forced on the 3x3 halo cases
# (ragged 21 x 37 and 'valid' 20 x 22 images, BN 64 / 128, Cout 48; x3.splitk's 8 x 8 image
# keeps the 8 x 16 patch), one patch per block and 3 per block; the fp64 bar, and bit-identity
# with the 8 x 16 patch -- each output's K-tiles and MFMAs run in the same order on both
X3_PH16_CASES = [(c, pt) for c in X3_CASES[:6] for pt in (None, 3)]


@gpu
@pytest.mark.parametrize("case,pt", X3_PH16_CASES, ids=[f"{c[0]}-pt{pt}" for c, pt in X3_PH16_CASES])
def test_x3_16x16_patch_matches_fp64_and_the_8x16_patch(case, pt, monkeypatch, capfd):
    monkeypatch.delenv("DG_PLAN_DISABLE", raising=False)
    if pt:
        monkeypatch.setenv("DG_X3H_PTILES", str(pt))
    monkeypatch.setenv("DG_X3H_PH", "16")
    monkeypatch.setenv("DG_PLAN_DEBUG", "1")
    test_conv_layer(case, "f16x3")
    name, N, H, W, Cin, Cout, k, s, padding, transpose, bias = case
    d16 = ops.ConvDesc(N, H, W, Cin, Cout, k, s, padding, transpose, math="f16x3")
    err = capfd.readouterr().err
    fwd_plan = [l for l in err.splitlines() if l.startswith("[dg plan] mode 0") and "x3h" in l][-1]
    assert (" ph 16 " in fwd_plan) == (H >= 16), fwd_plan
    monkeypatch.setenv("DG_X3H_PH", "8")
    d8 = ops.ConvDesc(N, H, W, Cin, Cout, k, s, padding, transpose, math="f16x3")
    x, w = _rand((N, H, W, Cin), 11), _rand(d16.weight_shape, 12, 0.05)
    dy = _rand(d16.out_shape, 13)
    ys = [torch.empty(d16.out_shape, device="cuda") for _ in range(2)]
    dxs = [torch.empty_like(x) for _ in range(2)]
    for d, y, dx in zip((d16, d8), ys, dxs):
        d.fwd(x, w, y)
        d.bwd_data(dy, w, dx)
    torch.cuda.synchronize()
    assert torch.equal(ys[0], ys[1]), f"{name}: forward differs between the 16x16 and 8x16 patches"
    assert torch.equal(dxs[0], dxs[1]), f"{name}: input gradient differs between the 16x16 and 8x16 patches"


@gpu
def test_x3_shared_weight_planes_serve_bwd_data():
    """One weight PlaneBuf: the fp16x3 forward splits it; the (fp16x3) input gradient reading
    it equals the one that splits w itself.  Every reader of w runs fp16x3 here, so the buffer
    holds no bf16x6 part (tensor_plane_bytes)."""
    N, H, W, Ci, Co = 2, 24, 32, 64, 128
    d = ops.ConvDesc(N, H, W, Ci, Co, 3, 1, "same", math="f16x3")
    d.set_act_scale(x=(ops.max_slot(device="cuda"),))   # held x planes: a plain max slot, measured
    x, w, dy = _rand((N, H, W, Ci), 1), _rand(d.weight_shape, 2, 0.05), _rand((N, H, W, Co), 3)
    P = ops.ConvPlanes.for_desc(d, x=True, dy=True, w=True)
    assert P.w is not None and 4 * 9 * Ci * Co <= P.w.buf.numel() < 10 * 9 * Ci * Co
    y0, y1 = torch.empty(N, H, W, Co, device="cuda"), torch.empty(N, H, W, Co, device="cuda")
    d.fwd(x, w, y0)
    d.fwd(x, w, y1, planes=P)
    assert P.w.ready
    dx0, dx1 = torch.empty_like(x), torch.empty_like(x)
    d.bwd_data(dy, w, dx0)
    d.bwd_data(dy, w, dx1, planes=P)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    assert torch.equal(dx0, dx1)


@gpu
@pytest.mark.parametrize("prod_math", ["bf16x6", "f16x3"])
def test_x3_producer_planes_equal_the_split(prod_math):
    """conv A (relu) -> conv B (fp16x3): A's epilogue writes B's x planes (out_format
    fp16x3) scaled from A's output bound (dg_conv_set_act_scale: max |x| measured, A's weight
    bound, max |bias|); B's forward on them is bit-identical to B splitting A's fp32 output
    with the same scale source, and A's epilogue measures max |y_A| (B's input)."""
    N, H, W, C0, C1, C2 = 2, 24, 40, 32, 64, 128
    a = ops.ConvDesc(N, H, W, C0, C1, 3, 1, "same", math=prod_math)
    b = ops.ConvDesc(N, H, W, C1, C2, 3, 1, "same", math="f16x3")
    x = _rand((N, H, W, C0), 4)
    wa, wb = _rand(a.weight_shape, 5, 0.08), _rand(b.weight_shape, 6, 0.05)
    ba = _rand((C1,), 7, 0.1)
    mx, wbd, ymx = ops.max_slot(device="cuda"), torch.zeros(2, device="cuda"), ops.max_slot(device="cuda")
    ops.absmax_set(x, mx)
    ops.weight_bound(wa, wbd[0:1], bias=ba, c_out=wbd[1:2])
    src = (mx, wbd[0:1], wbd[1:2])
    a.set_act_scale(y=src, y_max=ymx)
    b.set_act_scale(x=src)
    ya = torch.empty(N, H, W, C1, device="cuda")
    Pb = ops.ConvPlanes.for_desc(b, x=True)
    assert Pb.x.fmt == ops.PLANES_F16X3 and Pb.x.buf.numel() >= 4 * N * H * W * C1
    Pa = ops.ConvPlanes()
    Pa.fwd_out = Pb.x
    a.fwd(x, wa, ya, bias=ba, act="relu", planes=Pa)
    assert Pb.x.ready
    y_fed, y_own = torch.empty(N, H, W, C2, device="cuda"), torch.empty(N, H, W, C2, device="cuda")
    b.fwd(ya, wb, y_fed, planes=Pb)        # reads the producer's planes
    Po = ops.ConvPlanes.for_desc(b, x=True)
    b.fwd(ya, wb, y_own, planes=Po)        # splits ya itself (same source)
    torch.cuda.synchronize()
    assert torch.equal(y_fed, y_own)
    assert float(ymx.max()) == float(ya.abs().max())
    bound = float(mx.max()) * float(wbd[0]) + float(wbd[1])
    assert float(ya.abs().max()) <= bound


@gpu
@pytest.mark.parametrize("ptiles,ph", [("1", "8"), ("3", "8"), ("1", "16"), ("3", "16")])
def test_x3_fused_pool_planes_and_unfused_pool(ptiles, ph, monkeypatch):
    """An fp16x3 conv with its 2x2 max pool fused (pool_fusable) writes the next fp16x3
    conv's x planes; so does the unfused pool (dg_maxpool2_fwd_plf).  Both equal the
    consumer's own split, and the pooled values equal conv -> pool -- with one patch per
    block and with persistent blocks of 3 patches (their max |pooled| folded across patches),
    on the 8 x 16 and the 16 x 16 patch."""
    monkeypatch.setenv("DG_X3H_PTILES", ptiles)
    monkeypatch.setenv("DG_X3H_PH", ph)
    N, H, W, Ci, Co, Cn = 4, 32, 32, 64, 128, 128
    d = ops.ConvDesc(N, H, W, Ci, Co, 3, 1, "same", math="f16x3")
    nxt = ops.ConvDesc(N, H // 2, W // 2, Co, Cn, 3, 1, "same", math="f16x3")
    assert d.pool_fusable("relu")
    x, w, b = _rand((N, H, W, Ci), 8), _rand(d.weight_shape, 9, 0.06), _rand((Co,), 10, 0.1)
    wn = _rand(nxt.weight_shape, 11, 0.05)
    # the pooled planes' scale source: d's output bound (max |x|, d's weight bound, max |b|)
    mx, wbd, pmx = ops.max_slot(device="cuda"), torch.zeros(2, device="cuda"), ops.max_slot(device="cuda")
    ops.absmax_set(x, mx)
    ops.weight_bound(w, wbd[0:1], bias=b, c_out=wbd[1:2])
    src = (mx, wbd[0:1], wbd[1:2])
    d.set_act_scale(x=(ops.max_slot(device="cuda"),), y=src, y_max=pmx)
    nxt.set_act_scale(x=src)
    y = torch.empty(N, H, W, Co, device="cuda")
    d.fwd(x, w, y, bias=b, act="relu")
    py0 = torch.empty(N, H // 2, W // 2, Co, device="cuda")
    P0 = ops.ConvPlanes.for_desc(nxt, x=True)
    ops.maxpool2_fwd(y, py0, planes_out=P0.x, scale=src)
    py1 = torch.empty_like(py0)
    P1 = ops.ConvPlanes.for_desc(nxt, x=True)
    idx = torch.empty((N, H // 2, W // 2, Co), dtype=torch.uint8, device="cuda")
    d.fwd_pool(x, w, idx, bias=b, act="relu", pool_y=py1, pool_planes=P1.x)
    P2 = ops.ConvPlanes.for_desc(nxt, x=True)
    yo = [torch.empty(N, H // 2, W // 2, Cn, device="cuda") for _ in range(3)]
    nxt.fwd(py0, wn, yo[0], planes=P0)
    nxt.fwd(py1, wn, yo[1], planes=P1)
    nxt.fwd(py0, wn, yo[2], planes=P2)      # (splits py0 into P2)
    torch.cuda.synchronize()
    assert torch.equal(py0, py1)
    nb = 4 * N * (H // 2) * (W // 2) * Co
    assert torch.equal(P0.x.buf[:nb], P1.x.buf[:nb]) and torch.equal(P0.x.buf[:nb], P2.x.buf[:nb])
    assert torch.equal(yo[0], yo[1]) and torch.equal(yo[0], yo[2])
    assert float(pmx.max()) == float(py1.abs().max())   # the fused pool measured its output


@gpu
def test_x3_xmask_from_hi_plane_sign():
    """dg_conv_bwd_data_xmask on fp16x3 x planes: act' from the sign of the fp16 hi
    piece equals act' from the fp32 activation (relu and leaky relu)."""
    N, H, W, Ci, Co = 2, 16, 32, 64, 64
    d = ops.ConvDesc(N, H, W, Ci, Co, 3, 1, "same", math="f16x3")
    z = _rand((N, H, W, Ci), 12)
    z = torch.where(z > 0, z, 0.3 * z)            # a leaky relu output (signs on both sides)
    w, dy = _rand(d.weight_shape, 13, 0.05), _rand((N, H, W, Co), 14)
    P = ops.ConvPlanes.for_desc(d, x=True, w=True)
    y = torch.empty(N, H, W, Co, device="cuda")
    d.fwd(z, w, y, planes=P)                      # splits z into P.x (fp16x3)
    assert P.x.ready and P.x.fmt == ops.PLANES_F16X3
    for act in ("lrelu", "relu"):
        dx0, dx1 = torch.empty_like(z), torch.empty_like(z)
        d.bwd_data_masked(dy, w, dx0, z, act, alpha=0.3)
        d.bwd_data_xmask(dy, w, dx1, act, alpha=0.3, planes=P)
        torch.cuda.synchronize()
        assert torch.equal(dx0, dx1), act


@gpu
def test_vgg_content_loss_x3_vs_bf16x6():
    """The VGG19 content loss with its forward on fp16x3 against the all-bf16x6 network on
    the same weights and inputs: value to 1e-6 relative, input gradient to 1e-4 in relative
    L2 and of its scale elementwise (measured 1.1e-5: unconditioned, a ReLU / pool near-tie
    of the 16 layers may route differently -- a sanity bar against indexing errors; the
    mask-conditioned fp64 bars are test_sr_gpu.py's and test_step_gpu.py's)."""
    from dgan.sr_trainer import ContentLoss, VGGNetwork
    N, H, W = 2, 64, 64
    nets = []
    for vm in ("f16x3", "bf16x6"):
        v = VGGNetwork(seed=5, width=4, device=torch.device("cuda"))
        v.conv_math = vm
        nets.append(v)
    g, t = _rand((N, H, W, 3), 15).clamp(-1, 1), _rand((N, H, W, 3), 16).clamp(-1, 1)
    out = []
    for v in nets:
        cl = ContentLoss(v, N, H, W, torch.device("cuda"))
        ws = ops.Workspace()
        ws.get(cl.ws_bytes)
        val = cl.forward(g, t, ws=ws)[0].clone()
        dg = torch.zeros(N, H, W, 3, device="cuda")
        cl.backward(dg, beta=0.0, ws=ws)
        out.append((val, dg))
        if v.conv_math == "f16x3":
            assert any(d.plane_format(ops.TENSOR_X) == ops.PLANES_F16X3 for d in cl.fplan.desc.values())
    torch.cuda.synchronize()
    (v0, g0), (v1, g1) = out
    assert abs(float(v0) - float(v1)) <= 1e-6 * abs(float(v1))
    assert float((g0 - g1).norm()) <= 1e-4 * float(g1.norm())
    assert float((g0 - g1).abs().max()) <= 1e-4 * float(g1.abs().max())


@gpu
def test_x3_input_gradient_chain_with_scale_context():
    """Two fp16x3 layers (A -> relu -> B): B's input gradient writes A's fp16x3 dy planes
    scaled from (max |dy_B|, B's weight bound) and measures max |dy_A| by atomicMax; A's
    input gradient reads them with the same scale source.  Against torch fp64 at the conv
    engine's bar (two layers deep: K of both), and max |dy_A| equals the fp32 dy_A's."""
    from torch_ref import conv2d_ref
    N, H, W, C0, C1, C2 = 2, 16, 32, 64, 64, 128
    a = ops.ConvDesc(N, H, W, C0, C1, 3, 1, "same", math="f16x3")
    b = ops.ConvDesc(N, H, W, C1, C2, 3, 1, "same", math="f16x3")
    for d in (a, b):
        assert d.plane_format(ops.TENSOR_DY) == ops.PLANES_F16X3
    x64 = torch.randn(N, H, W, C0, dtype=torch.float64)
    wa64 = torch.randn(*a.weight_shape, dtype=torch.float64) * 0.05
    wb64 = torch.randn(*b.weight_shape, dtype=torch.float64) * 0.05
    dy64 = torch.randn(N, H, W, C2, dtype=torch.float64) * 1e-7   # a small gradient (no static range)
    dev = torch.device("cuda")
    x, wa, wb, dy = (t.float().to(dev) for t in (x64, wa64, wb64, dy64))
    zA = torch.empty(N, H, W, C1, device=dev)
    a.fwd(x, wa, zA, act="relu")
    # the reference takes the GPU's relu decisions (an fp32 / fp64 near-tie would route differently)
    mask = (zA > 0).double().cpu()
    xr = x64.clone().requires_grad_()
    za = conv2d_ref(xr, wa64, 1, a.pads, None) * mask
    yb = conv2d_ref(za, wb64, 1, b.pads, None)
    yb.backward(dy64)
    gmax = ops.max_slot(2, device=dev)   # [A, B] max slots
    gwb = torch.stack([wa.abs().sum(dim=(0, 1, 3)).amax(), wb.abs().sum(dim=(0, 1, 3)).amax()])
    b.set_grad_scale(dy_m=gmax[1], dx_m=gmax[1], dx_g=gwb[1:2], dx_max=gmax[0])
    a.set_grad_scale(dy_m=gmax[1], dy_g=gwb[1:2])
    ops.absmax(dy, gmax[1])
    Pb, Pa = ops.ConvPlanes(), ops.ConvPlanes.for_desc(a, dy=True)
    assert Pa.dy.fmt == ops.PLANES_F16X3
    Pb.bwd_out = Pa.dy
    dzA = torch.empty(N, H, W, C1, device=dev)
    b.bwd_data_masked(dy, wb, dzA, zA, "relu", planes=Pb)        # writes A's dy planes
    assert Pa.dy.ready
    dx = torch.empty(N, H, W, C0, device=dev)
    a.bwd_data(dzA, wa, dx, planes=Pa)                            # reads them
    torch.cuda.synchronize()
    assert float(gmax[0].max()) == float(dzA.abs().max())
    assert float(gmax[1].max()) == float(dy.abs().max())
    _close(dx, xr.grad, 2 * 9 * max(C1, C2), "chain dx")


@gpu
@pytest.mark.parametrize("math", ["f16x3", "bf16x6"])
@pytest.mark.parametrize("Co", [128, 512])
def test_bwd_data_masked_sum(math, Co):
    """dg_conv_bwd_data_masked_sum: dx = act'(z) * (dL/dx + beta dx) -- the U-Net's down1
    gradient fan-in (skip + down2) masked once after the sum -- equals act'(z) applied in torch to
    the unmasked input gradient plus the prior dx, on the halo phases kernel's epilogue and (the
    K of 512 output channels splits) through the split-K reduce."""
    N, H, W, Ci = 2, 32, 32, 64
    d = ops.ConvDesc(N, H, W, Ci, Co, 4, 2, "same", math=math)
    w, dy = _rand(d.weight_shape, 21, 0.05), _rand(d.out_shape, 22)
    z = _rand((N, H, W, Ci), 23)
    prior = _rand((N, H, W, Ci), 24)
    dx = prior.clone()
    if d.op_arith("bwd_data") == "fp32":   # (the planner kept this size on fp32 tiles: refused, loudly)
        with pytest.raises(ops.DGError, match="split-precision"):
            d.bwd_data_masked_sum(dy, w, dx, z, "lrelu", 0.3, beta=1.0)
        return
    dx_plain = torch.empty(N, H, W, Ci, device="cuda")
    d.bwd_data(dy, w, dx_plain)
    d.bwd_data_masked_sum(dy, w, dx, z, "lrelu", 0.3, beta=1.0)
    torch.cuda.synchronize()
    mask = torch.where(z > 0, torch.ones_like(z), torch.full_like(z, 0.3))
    ref = mask * (dx_plain + prior)
    err = (dx - ref).abs().max().item()
    assert err <= 2e-6 * ref.abs().max().item(), err
