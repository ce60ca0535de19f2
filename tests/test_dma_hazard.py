"""Audit of the shipped code objects for the LDS-DMA wait-state hazards (CPU: disassembles
denoise-gan_amd/lib/libdgan.so with the ROCm LLVM tools; no GPU).

The GEMM kernels issue their global -> LDS copies (`buffer_load_dwordx4 ... offen lds`) from an
inline-asm statement (csrc/conv_x6.h dma16), and hipcc pads no hazard into an asm statement
(cdna_hip_programming.md §5.7 item 2).  Two hazards reach it: a VALU write of an SGPR of the buffer
descriptor (hipcc's SGPR-spill restores, `v_readlane_b32`) needs 5 wait states before the VMEM
instruction reads it, and the `s_mov_b32 m0` hipcc writes for the DMA's LDS address one.  In round
6 a register-allocation change put a restore two instructions ahead of a DMA of the fp16x3 KT 2
halo kernel: the generator's forward differed run to run and one run faulted the GPU
(scripts/diag/determinism.py).  The asm now opens with `s_nop 4`; this test holds every LDS-DMA
of the library to that pad, and to >= 5 wait states after any VALU write of its descriptor SGPRs.
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(REPO, "denoise-gan_amd", "lib", "libdgan.so")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tools_ok():
    return all(os.path.exists(os.path.join(LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump"))


def _disassemble(tmp):
    fb = os.path.join(tmp, "fatbin")
    subprocess.run([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", f".hip_fatbin={fb}", LIB, os.path.join(tmp, "lib.so")],
                   check=True, capture_output=True)
    data = open(fb, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    for i, s in enumerate(starts):
        chunk = os.path.join(tmp, f"b{i}")
        with open(chunk, "wb") as f:
            f.write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
        dev = os.path.join(tmp, f"d{i}.o")
        r = subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={chunk}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], capture_output=True)
        if r.returncode or not os.path.getsize(dev):
            continue
        d = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", dev], check=True,
                           capture_output=True, text=True)
        out.append(d.stdout)
    return out


def _instrs(text):
    """[(function, instruction text)] in program order."""
    fn, out = None, []
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            fn = m.group(1)
            continue
        s = line.strip()
        if not s or s.startswith(";") or s.endswith(":") or fn is None:
            continue
        out.append((fn, s.split("//")[0].strip()))
    return out


@pytest.mark.skipif(not (os.path.exists(LIB) and _tools_ok()), reason="library or ROCm LLVM tools missing")
def test_every_lds_dma_is_padded(tmp_path):
    texts = _disassemble(str(tmp_path))
    assert texts, "no gfx950 code object in the library"
    n_dma, bad = 0, []
    for text in texts:
        ins = _instrs(text)
        for i, (fn, s) in enumerate(ins):
            if not (s.startswith("buffer_load_dwordx4") and s.endswith(" lds") or " lds" in s and s.startswith("buffer_load")):
                continue
            n_dma += 1
            prev = ins[i - 1][1] if i else ""
            m = re.match(r"s_nop (\d+)", prev)
            if not m or int(m.group(1)) < 4:
                bad.append((fn[:80], prev, s))
                continue
            # >= 5 wait states between a VALU write of a descriptor SGPR and the DMA
            d = re.search(r"s\[(\d+):(\d+)\]", s)
            regs = set(range(int(d.group(1)), int(d.group(2)) + 1)) if d else set()
            waits = 0
            for j in range(i - 1, max(-1, i - 12), -1):
                p = ins[j][1]
                if ins[j][0] != fn:
                    break
                w = re.match(r"s_nop (\d+)", p)
                v = re.match(r"v_\w+\s+s(\d+)", p)
                if v and int(v.group(1)) in regs and waits < 5:
                    bad.append((fn[:80], p, s))
                    break
                waits += int(w.group(1)) + 1 if w else 1
                if waits >= 5:
                    break
    assert n_dma > 1000, f"only {n_dma} LDS-DMA instructions found"
    assert not bad, f"{len(bad)} LDS-DMAs without their wait states, e.g. {bad[:3]}"
