"""Loading and comparing the committed golden fixtures (tests/golden/*.npz,
written by scripts/gen_golden.py from the fp64 oracles)."""
import json
import math
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "scripts"))


def load(case):
    path = os.path.join(GOLDEN, case + ".npz")
    with np.load(path, allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    meta = json.loads(str(d.pop("meta")))
    return meta, d


def batch(meta, seed):
    from gen_golden import batch as _b
    return _b(meta, seed)


def weights_crc(params, order):
    c = 0
    for n in order:
        c = zlib.crc32(np.ascontiguousarray(params[n], np.float32).tobytes(), c)
    return c


def psnr(img, ref):
    a = (np.asarray(img, np.float64) + 1) / 2
    b = (np.asarray(ref, np.float64) + 1) / 2
    return 10 * math.log10(1.0 / np.mean((a - b) ** 2))


def names(d, prefix):
    """variable names digested under prefix (e.g. 's1|gG|')."""
    return sorted({k[len(prefix):].rsplit("|", 1)[0] for k in d if k.startswith(prefix)})


def compare_digest(d, prefix, values, atol, l2_rtol=None, what="", rel=0.0):
    """values: name -> array.  Sampled entries to max-abs atol (+ rel * the variable's max |ref|);
    the L2 norm to l2_rtol.  Returns the worst (err, name)."""
    worst = (0.0, None)
    for n in names(d, prefix):
        flat = np.asarray(values[n], np.float64).ravel()
        idx = d[f"{prefix}{n}|idx"]
        err = float(np.abs(flat[idx] - d[f"{prefix}{n}|val"]).max())
        tol = atol + rel * float(d.get(f"{prefix}{n}|maxabs", 0.0))
        assert err <= tol, f"{what} {n}: sampled max-abs diff {err:.3e} > {tol:.1e}"
        if l2_rtol is not None:
            ref = float(d[f"{prefix}{n}|l2"])
            l2rel = abs(float(np.linalg.norm(flat)) - ref) / max(ref, 1e-30)
            assert l2rel <= l2_rtol or abs(float(np.linalg.norm(flat)) - ref) <= atol, \
                f"{what} {n}: L2 norm {np.linalg.norm(flat):.6e} vs {ref:.6e}"
        if err > worst[0]:
            worst = (err, n)
    return worst
