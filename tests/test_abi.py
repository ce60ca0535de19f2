"""The C-ABI library (no GPU needed): it builds for gfx950, loads, exports
every entry point declared in include/dgan.h with the argument list the
ctypes binding uses, and the host-side geometry helpers restate TF's rules."""
import os
import re
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dgan.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|const char \*)\s*\*?\s*(dg_[a-z0-9_]+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(1)] = args
    return out


def test_library_builds_and_exports_every_declared_symbol():
    import dgan
    from dgan import _lib
    path = dgan.build()
    assert os.path.exists(path)
    nm = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (dg_[a-z0-9_]+)", nm))
    decl = _declared()
    assert len(decl) >= 20
    missing = sorted(set(decl) - exported)
    assert not missing, f"declared but not exported: {missing}"
    L = _lib.lib()
    for name in decl:
        assert hasattr(L, name)


def test_loaded_binary_is_built_from_this_tree():
    """Binary provenance: the library carries the hash of the sources it was compiled from
    (dg_build_info, dgan/build.py), and it is this tree's -- the GPU suite and the bench load
    this same in-tree file."""
    from dgan import _lib
    from dgan.build import source_sha
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    from pmc_traffic import csrc_sha
    info = _lib.build_info()
    assert info["source_sha"] == source_sha() == csrc_sha(), info
    assert info["arch"] == "gfx950"


def test_ctypes_signatures_match_header_arity():
    from dgan import _lib
    decl = _declared()
    assert set(decl) == set(_lib.EXPORTED)
    for name, args in decl.items():
        assert len(_lib._SIGS[name][1]) == len(args), name


def test_library_loads_without_gpu_and_reports_errors():
    import ctypes
    from dgan import _lib
    L = _lib.lib()
    assert L.dg_version() == 1
    from dgan import ops
    assert L.dg_max_slot_floats() == ops.MAX_SLOT == 256   # include/dgan.h DG_MAX_SLOT
    h = ctypes.c_void_p()
    rc = L.dg_conv_desc_create(ctypes.byref(h), 0, 8, 8, 4, 4, 3, 3, 1, 1, 1, 1, 1, 1, 0)
    assert rc != 0
    assert b"bad shape" in L.dg_last_error_string()


def test_conv_descriptor_geometry_and_workspace():
    from dgan.ops import ConvDesc, tf_same_pads
    d = ConvDesc(16, 256, 256, 3, 64, 4, 2, "same")
    assert (d.Ho, d.Wo) == (128, 128) and d.pads == (1, 1, 1, 1)
    t = ConvDesc(16, 128, 128, 128, 3, 4, 2, "same", transpose=True)
    assert (t.Ho, t.Wo) == (256, 256) and t.pads == (1, 1, 1, 1)
    assert t.weight_shape == (4, 4, 3, 128)
    v = ConvDesc(16, 32, 32, 256, 512, 4, 1, (1, 1, 1, 1))
    assert (v.Ho, v.Wo) == (31, 31)
    a = ConvDesc(2, 12, 12, 32, 64, 3, 2, "same")
    assert a.pads == (0, 1, 0, 1) and (a.Ho, a.Wo) == (6, 6)
    assert tf_same_pads(256, 4, 2) == (1, 1)
    # deep layers are split-K: they need slab workspace, and every query is consistent
    deep = ConvDesc(16, 2, 2, 512, 512, 4, 2, "same")
    assert deep.ws[0] > 0 and all(w >= 0 for w in deep.ws)
    assert d.flops == 2 * 16 * 128 * 128 * 64 * 16 * 3


def test_gpu_ops_fail_loudly_without_device():
    import torch
    from dgan import ops
    d = ops.ConvDesc(1, 8, 8, 32, 32, 4, 2, "same")
    x = torch.zeros(1, 8, 8, 32)
    with pytest.raises(ops.DGError):
        d.fwd(x, torch.zeros(d.weight_shape), torch.zeros(d.out_shape))
