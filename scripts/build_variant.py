#!/usr/bin/env python3
"""Build a variant of libdgan.so with extra compile flags, for same-box A/B:

    python scripts/build_variant.py NAME -DDG_X6_DEFER=1 ...
    -> denoise-gan_amd/lib/libdgan_NAME.so   (load it with DG_LIB=<path>)"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "denoise-gan_amd"))
os.environ.pop("DG_LIB", None)
import importlib  # noqa: E402
B = importlib.import_module("dgan.build")


def main(name, flags):
    obj = os.path.join(B.LIBDIR, f"obj_{name}")
    os.makedirs(obj, exist_ok=True)
    srcs = B._sources()

    def one(f):
        o = os.path.join(obj, f[:-4] + ".o")
        r = subprocess.run([B.HIPCC] + B.CXXFLAGS + flags + ["-c", os.path.join(B.CSRC, f), "-o", o],
                           capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr)
        return o

    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(one, srcs))
    lib = os.path.join(B.LIBDIR, f"libdgan_{name}.so")
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", lib] + objs, check=True)
    print(lib)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
