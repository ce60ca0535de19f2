"""Host-side planner choices for the bs16 training step's conv layers (no GPU:
descriptors are planned at creation).  Pins the kernel family each pix2pix
layer op runs on (csrc/conv.hip make_plan / plan_recast, printed under
DG_PLAN_DEBUG), so a planner change that silently moves a layer back to a
slower path shows up here; the GPU tests hold every path to the fp64 bar."""
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "denoise-gan_amd", "lib", "libdgan.so")

# (layer, N, H, W, Cin, Cout, k, s, padding, transpose) of the batched 2N = 32 passes
LAYERS = {
    "D.last": (32, 31, 31, 512, 1, 4, 1, (1, 1, 1, 1), False),
    "D.conv": (32, 32, 32, 256, 512, 4, 1, (1, 1, 1, 1), False),
    "G.last": (32, 128, 128, 128, 3, 4, 2, "same", True),
    "G.up7": (32, 64, 64, 256, 64, 4, 2, "same", True),
    "G.down1": (32, 256, 256, 3, 64, 4, 2, "same", False),
    "V.b3c2": (32, 64, 64, 256, 256, 3, 1, "same", False),
    # SRGAN's VGG19 under mixed_float16 (bs32: generated + real batches, 96^2)
    "S.vgg_f16": (64, 96, 96, 128, 128, 3, 1, "same", False, "fp16"),
    "S.res_f16": (32, 24, 24, 64, 64, 3, 1, "same", False, "fp16"),
}

SCRIPT = r"""
import sys
sys.path[:0] = [sys.argv[1]]
from dgan.ops import ConvDesc
N, H, W, ci, co, k, s, pad, tr, *math = eval(sys.argv[2])
ConvDesc(N, H, W, ci, co, k, s, pad, tr, math=math[0] if math else None)
"""


def _plans(spec):
    env = dict(os.environ, DG_PLAN_DEBUG="1")
    env.pop("DG_PLAN_DISABLE", None)
    r = subprocess.run([sys.executable, "-c", SCRIPT, os.path.join(REPO, "denoise-gan_amd"), repr(spec)],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    return re.findall(r"\[dg plan\] mode (\d)[^>]*-> (\w+)", r.stderr)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libdgan.so not built")
@pytest.mark.parametrize("layer,expect", [
    # Co == 1 head: input and filter gradients on the direct kernels (the forward recast is
    # a 1x1 GEMM planned as a second descriptor)
    ("D.last", {"1": "co1", "2": "co1"}),
    # the PatchGAN conv's input gradient on the stride-1 4x4 halo tiles
    ("D.conv", {"1": "x6h4"}),
    # Conv2DTranspose(3) forward = conv-view DGRAD on the fused MFMA + col2im kernel
    ("G.last", {"1": "tlast"}),
    # ConvT(64) forward on the stride-2 phase halo
    ("G.up7", {"1": "x6h2"}),
    # Cin 3: small-Cin strip kernels for forward and filter gradient
    ("G.down1", {"0": "small", "2": "small"}),
    # VGG19 3x3: halo tiles both ways
    ("V.b3c2", {"0": "x6h", "1": "x6h"}),
    # fp16 3x3 stride 1 (32-channel chunks): the halo tiles' fp16 variant both ways
    ("S.vgg_f16", {"0": "f16h", "1": "f16h"}),
    ("S.res_f16", {"0": "f16h", "1": "f16h"}),
])
def test_plan_kernel_family(layer, expect):
    got = {}
    for mode, kind in _plans(LAYERS[layer]):
        if len(LAYERS[layer]) > 9:
            got[mode] = kind   # a math= descriptor plans the default math first, its own last
        else:
            got.setdefault(mode, kind)
    for mode, kind in expect.items():
        assert got.get(mode) == kind, (layer, got)


CSRC = os.path.join(REPO, "denoise-gan_amd", "csrc")


def test_no_plan_choice_justified_by_a_fixture():
    """Kernel selection follows same-box timing, never a test outcome: no csrc/ source may
    justify a plan choice by a golden fixture (the fixtures are drift pins, tests/test_golden_gpu.py)."""
    bad = []
    for f in sorted(os.listdir(CSRC)):
        with open(os.path.join(CSRC, f)) as fh:
            for i, line in enumerate(fh, 1):
                if re.search(r"golden|fixture", line, re.I):
                    bad.append(f"{f}:{i}: {line.strip()}")
    assert not bad, bad


def test_size_thresholds_cite_a_measurement():
    """Every named size threshold of the planner (constexpr ... _MIN_ / _MAX_ in csrc/) is preceded by
    a comment citing the A/B that set it, and the cited profile is committed."""
    for f in sorted(os.listdir(CSRC)):
        lines = open(os.path.join(CSRC, f)).read().split("\n")
        for i, line in enumerate(lines):
            m = re.match(r"\s*constexpr\s+\w+\s+(\w*_MIN_\w*|\w*_MAX_\w*)\s*=", line)
            if not m:
                continue
            j = i - 1
            block = []
            while j >= 0 and lines[j].strip().startswith("//"):
                block.append(lines[j])
                j -= 1
            text = " ".join(block)
            assert re.search(r"A/B|measured|sweep", text), (f, m.group(1))
            for ref in re.findall(r"profiles/[\w/.\-]+", text):
                assert os.path.exists(os.path.join(REPO, ref.rstrip(".,)"))), (f, m.group(1), ref)
