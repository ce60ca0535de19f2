"""Build libdgan.so (gfx950) from csrc/*.hip with hipcc.

Incremental: an object is rebuilt when its source, common.h or dgan.h is
newer.  Objects and the library stay in-tree (denoise-gan_amd/lib) so they
travel to the GPU box with the repository snapshot.
"""
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


def _newer(src_paths, dst):
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(p) > t for p in src_paths)


def build(verbose=False, jobs=None):
    if os.environ.get("DG_LIB"):
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"DG_LIB={LIB_PATH} does not exist")
        return LIB_PATH
    os.makedirs(OBJDIR, exist_ok=True)
    deps = [os.path.join(CSRC, h) for h in os.listdir(CSRC) if h.endswith(".h")] + [os.path.join(INCLUDE, "dgan.h")]
    todo = []
    objs = []
    for f in _sources():
        src = os.path.join(CSRC, f)
        obj = os.path.join(OBJDIR, f[:-4] + ".o")
        objs.append(obj)
        if _newer([src] + deps, obj):
            todo.append((src, obj))

    def compile_one(item):
        src, obj = item
        cmd = [HIPCC] + CXXFLAGS + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
        return obj

    if todo:
        n = jobs or min(len(todo), max(1, (os.cpu_count() or 4) // 2), 8)
        with ThreadPoolExecutor(max_workers=n) as ex:
            list(ex.map(compile_one, todo))
    if todo or _newer(objs, LIB_PATH):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB_PATH] + objs
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB_PATH


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
