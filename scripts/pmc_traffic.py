#!/usr/bin/env python3
"""Per-step HBM bytes of the conv-engine kernels from two rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE; kilobytes per dispatch).  FETCH_SIZE is
doubled: on gfx950 it reports half the bytes of 16-B-per-lane streaming
reads (MI355X_MICROARCH.md, HBM section), the access width of the conv
engine's operand loads (buffer_load ... lds dwordx4) and split passes.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV STEPS [OUT_JSON [PROFILE_LABEL [COMMIT]]]

The JSON carries csrc_sha (csrc_sha() of the measured tree)."""
import csv
import hashlib
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def csrc_sha():
    """sha256 over the library sources (denoise-gan_amd/csrc/*, include/dgan.h): the stamp that
    ties a committed traffic profile to the kernels it measured (tests/test_profiles.py)."""
    h = hashlib.sha256()
    csrc = os.path.join(REPO, "denoise-gan_amd", "csrc")
    for path in [os.path.join(csrc, f) for f in sorted(os.listdir(csrc))] + [os.path.join(REPO, "include", "dgan.h")]:
        h.update(os.path.basename(path).encode())
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]

CONV = ("k_conv_gemm", "k_split3", "k_splitk_reduce", "k_narrow", "k_direct", "k_recast", "k_transpose", "k_colsum",
        "k_small", "k_co1", "k_tlast")


def load(path, counter):
    per = defaultdict(float)
    n = defaultdict(int)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"]
            per[k] += float(r["Counter_Value"]) * 1024.0
            n[k] += 1
    return per, n


METHOD = ("rocprofv3 --pmc FETCH_SIZE (x2, gfx950 16B/lane correction) and --pmc WRITE_SIZE in separate "
          "passes over bench.py --profile-only --no-graph; kernels " + ", ".join(CONV))


def summarise(fetch_csv, write_csv, steps):
    """Per-step conv-engine HBM bytes of two PMC passes over `steps` training steps."""
    fe, _ = load(fetch_csv, "FETCH_SIZE")
    wr, _ = load(write_csv, "WRITE_SIZE")
    tot_f = sum(v for k, v in fe.items() if any(c in k for c in CONV)) * 2.0
    tot_w = sum(v for k, v in wr.items() if any(c in k for c in CONV))
    return {"conv_engine_bytes_per_step": (tot_f + tot_w) / steps, "read_bytes_per_step": tot_f / steps,
            "write_bytes_per_step": tot_w / steps, "steps": steps, "method": METHOD, "csrc_sha": csrc_sha()}


def main(fetch_csv, write_csv, steps, out_json=None, profile=None, commit=None):
    steps = int(steps)
    fe, _ = load(fetch_csv, "FETCH_SIZE")
    wr, _ = load(write_csv, "WRITE_SIZE")
    tot_f = sum(v for k, v in fe.items() if any(c in k for c in CONV)) * 2.0
    tot_w = sum(v for k, v in wr.items() if any(c in k for c in CONV))
    print(f"conv engine HBM bytes/step: read {tot_f / steps / 1e9:.3f} GB (FETCH_SIZE x2), "
          f"write {tot_w / steps / 1e9:.3f} GB, total {(tot_f + tot_w) / steps / 1e9:.3f} GB")
    rows = defaultdict(lambda: [0.0, 0.0])
    for k, v in fe.items():
        rows[k.split("(")[0][-60:]][0] += 2 * v / steps
    for k, v in wr.items():
        rows[k.split("(")[0][-60:]][1] += v / steps
    for k, (f, w) in sorted(rows.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))[:25]:
        print(f"  {k:60s} read {f / 1e9:8.3f} GB  write {w / 1e9:8.3f} GB")
    if out_json:
        t = summarise(fetch_csv, write_csv, steps)
        t["profile"] = profile
        t["commit"] = commit
        with open(out_json, "w") as f:
            json.dump(t, f, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:7])
