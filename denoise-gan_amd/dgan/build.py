"""Build libdgan.so (gfx950) from csrc/*.hip with hipcc.

Incremental by content: an object is rebuilt when the hash of its source, the
shared headers (csrc/*.h, include/dgan.h) and the compile flags differs from
the hash it was built from (a `.stamp` beside each object).  runtime.hip is
compiled with DG_SOURCE_SHA = the hash of every library source
(`source_sha()`, the same stamp the committed traffic profiles carry), so
`dg_build_info()` of a loaded binary names the sources it was built from
(tests/test_abi.py checks it against the tree; bench.py prints it).  Objects
and the library stay in-tree (denoise-gan_amd/lib) so they travel to the GPU
box with the repository snapshot.
"""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # denoise-gan_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
CSRC = os.path.join(PKG_ROOT, "csrc")
LIBDIR = os.path.join(PKG_ROOT, "lib")
OBJDIR = os.path.join(LIBDIR, "obj")
INCLUDE = os.path.join(REPO_ROOT, "include")
# DG_LIB: load a prebuilt variant library instead (A/B runs on one box); build() then builds nothing
LIB_PATH = os.environ.get("DG_LIB") or os.path.join(LIBDIR, "libdgan.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I" + INCLUDE, "-I" + CSRC,
            "-Wno-unused-result"]


def _sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


def source_sha(csrc=CSRC, header=os.path.join(INCLUDE, "dgan.h")):
    """sha256 (16 hex digits) over the library sources: every file of csrc/ in name order and
    include/dgan.h, each as (basename, bytes) -- scripts/pmc_traffic.csrc_sha."""
    h = hashlib.sha256()
    for path in [os.path.join(csrc, f) for f in sorted(os.listdir(csrc))] + [header]:
        h.update(os.path.basename(path).encode())
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _digest(paths, flags):
    """Content hash of files (by repository-relative name) and flags (the repository path
    written as '.'): the same tree gives the same digest here and on the GPU box, which
    runs the snapshot from another directory."""
    h = hashlib.sha256()
    for p in paths:
        h.update(os.path.relpath(p, REPO_ROOT).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).replace(REPO_ROOT, ".").encode())
    return h.hexdigest()


def _stamp_ok(obj, digest):
    st = obj + ".stamp"
    return os.path.exists(obj) and os.path.exists(st) and open(st).read().strip() == digest


def build(verbose=False, jobs=None):
    if os.environ.get("DG_LIB"):
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"DG_LIB={LIB_PATH} does not exist")
        return LIB_PATH
    deps = sorted([os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")] +
                  [os.path.join(INCLUDE, "dgan.h")])
    sha = source_sha()
    # the library's own stamp: every source and the flags it was built from (the GPU box gets the
    # library and this stamp with the snapshot, not the objects: a current library is not rebuilt)
    lib_digest = _digest([os.path.join(CSRC, f) for f in _sources()] + deps, CXXFLAGS + [ARCH, sha])
    if _stamp_ok(LIB_PATH, lib_digest):
        return LIB_PATH
    os.makedirs(OBJDIR, exist_ok=True)
    todo = []
    objs = []
    for f in _sources():
        src = os.path.join(CSRC, f)
        obj = os.path.join(OBJDIR, f[:-4] + ".o")
        flags = CXXFLAGS + ([f'-DDG_SOURCE_SHA="{sha}"'] if f == "runtime.hip" else [])
        digest = _digest([src] + deps, flags)
        objs.append(obj)
        if not _stamp_ok(obj, digest):
            todo.append((src, obj, flags, digest))

    def compile_one(item):
        src, obj, flags, digest = item
        cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        with open(obj + ".stamp", "w") as fh:
            fh.write(digest + "\n")
        return obj

    if todo:
        n = jobs or min(len(todo), max(1, (os.cpu_count() or 4) // 2), 8)
        with ThreadPoolExecutor(max_workers=n) as ex:
            list(ex.map(compile_one, todo))
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB_PATH] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    with open(LIB_PATH + ".stamp", "w") as fh:
        fh.write(lib_digest + "\n")
    return LIB_PATH


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
