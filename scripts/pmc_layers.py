#!/usr/bin/env python3
"""Per-conv-call HBM traffic of one training step from per-dispatch rocprofv3 PMC
counters, against each call's algorithmic bytes (x, w and y once each, fp32).

Two modes:

  run    one step of a BASELINE workload with every conv call bracketed by dg_mark
         dispatches (ops.ConvProfile(markers=True)); writes the mark sequence and
         the conv records to --out (JSON).  Run it under rocprofv3, once per counter
         (FETCH_SIZE and WRITE_SIZE do not fit one pass):
           rocprofv3 --pmc FETCH_SIZE -d D -o pmc --output-format csv -- \\
               python3 scripts/pmc_layers.py run --out marks.json
  table  attribute every dispatch of the marked step: a dispatch between the begin
         and end marks of conv call i belongs to that call (its GEMM, split passes,
         split-K reduce); the others are grouped by kernel name.  FETCH_SIZE is
         doubled (gfx950: it reports half the bytes of 16-B-per-lane streaming reads,
         MI355X_MICROARCH.md HBM section).  Prints a markdown table headed by the
         csrc_sha of the measured tree:
           python scripts/pmc_layers.py table --fetch F.csv --write W.csv --marks marks.json
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "denoise-gan_amd"), REPO, os.path.join(REPO, "scripts")]


def run(a):
    import torch
    from bench import Args, WORKLOADS, synthetic_batch
    from dgan import ops
    wl = WORKLOADS[a.model]
    batch = a.batch or wl["batch"]
    if a.model == "pix2pix":
        from pix2pix import Pix2Pix
        m = Pix2Pix(Args(crop_size=wl["size"], retrain=0, width=1, seed=1234, dropout_seed=0, identity_loss=1,
                         content_loss=int(not a.no_content)))
    else:
        from autoencoder import Autoencoder
        from fsrgan import FastSRGAN
        from srgan import SRGAN
        cls = {"srgan": SRGAN, "fsrgan": FastSRGAN, "autoencoder": Autoencoder}[a.model]
        fp16 = int(wl.get("fp16", 0) if a.fp16 is None else a.fp16)
        m = cls(Args(crop_size=wl["size"], scale=wl["scale"], lr=1e-3, fp16=fp16, retrain=0, seed=1234,
                     content_loss=int(not a.no_content)))
    x, y = (torch.from_numpy(t).cuda() for t in synthetic_batch(wl, batch, 1000))
    tr = m.trainer(x.shape) if a.model == "pix2pix" else m.trainer(x.shape, y.shape)
    for _ in range(2):
        tr.step(x, y)
    torch.cuda.synchronize()
    with ops.ConvProfile(markers=True) as prof:
        prof.mark("step_begin")
        tr.step(x, y)
        prof.mark("step_end")
    torch.cuda.synchronize()
    recs = [dict(label=r["label"], op=r["op"], shape=r["shape"], flops=r["flops"], bytes=r["bytes"])
            for r in prof.summary()]
    with open(a.out, "w") as f:
        json.dump({"model": a.model, "batch": batch, "marks": prof.marks, "records": recs}, f)


def _load(path, counter):
    """[(dispatch id, kernel name, value bytes)] in dispatch order (path: the CSV, or a
    rocprofv3 -d directory holding one *counter_collection.csv)."""
    if os.path.isdir(path):
        found = [os.path.join(r, f) for r, _, fs in os.walk(path) for f in fs if f.endswith("counter_collection.csv")]
        if len(found) != 1:
            raise SystemExit(f"{path}: {len(found)} counter_collection.csv files")
        path = found[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0))
    rows.sort()
    return rows


def _short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").strip()[-70:]


def attribute(rows, marks):
    """{key: bytes} over the marked step: key ("conv", i) or ("other", kernel)."""
    mi = [i for i, (_, k, _) in enumerate(rows) if "k_mark" in k]
    if len(mi) < len(marks):
        raise SystemExit(f"{len(mi)} mark dispatches in the trace, {len(marks)} expected")
    mi = mi[-len(marks):]   # (the marked step is the run's last; earlier marks: none)
    out = defaultdict(float)
    cur = None
    for j in range(len(mi) - 1):
        kind = marks[j]
        if isinstance(kind, list) and kind[0] == "begin":
            cur = ("conv", kind[1])
        elif isinstance(kind, list) and kind[0] == "end":
            cur = None
        elif kind == "step_end":
            break
        for i in range(mi[j] + 1, mi[j + 1]):
            _, k, v = rows[i]
            out[cur if cur is not None else ("other", _short(k))] += v
    return out


def table(a):
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    from pmc_traffic import csrc_sha
    meta = json.load(open(a.marks))
    marks, recs = meta["marks"], meta["records"]
    fe = attribute(_load(a.fetch, "FETCH_SIZE"), marks)
    wr = attribute(_load(a.write, "WRITE_SIZE"), marks)
    keys = set(fe) | set(wr)
    per_layer = defaultdict(lambda: [0, 0.0, 0.0, 0.0])   # (net, layer, op) -> calls, alg, read, write
    for k in keys:
        if k[0] != "conv":
            continue
        r = recs[k[1]]
        lab = r["label"] or "?.?"
        net, layer = lab.split(".", 1)
        e = per_layer[(net, layer, r["op"], tuple(r["shape"]))]
        e[0] += 1
        e[1] += r["bytes"]
        e[2] += 2.0 * fe.get(k, 0.0)
        e[3] += wr.get(k, 0.0)
    other = defaultdict(lambda: [0.0, 0.0])
    for k in keys:
        if k[0] == "other":
            other[k[1]][0] += 2.0 * fe.get(k, 0.0)
            other[k[1]][1] += wr.get(k, 0.0)
    tot_alg = sum(e[1] for e in per_layer.values())
    tot_rd = sum(e[2] for e in per_layer.values())
    tot_wr = sum(e[3] for e in per_layer.values())
    print(f"# Per-conv-call HBM traffic, {meta['model']} bs{meta['batch']}, one training step")
    print()
    print(f"csrc_sha {csrc_sha()} (scripts/pmc_traffic.py); rocprofv3 --pmc FETCH_SIZE (x2, gfx950 16-B/lane "
          f"correction) and WRITE_SIZE in separate passes over `scripts/pmc_layers.py run`; every dispatch between "
          f"a conv call's two dg_mark dispatches is that call's (GEMM, split passes, split-K reduce).")
    print()
    print(f"- conv calls: algorithmic {tot_alg / 1e9:.2f} GB, measured read {tot_rd / 1e9:.2f} GB + write "
          f"{tot_wr / 1e9:.2f} GB = {(tot_rd + tot_wr) / 1e9:.2f} GB ({(tot_rd + tot_wr) / max(tot_alg, 1):.2f}x)")
    oth = sum(v[0] + v[1] for v in other.values())
    print(f"- other kernels of the step: {oth / 1e9:.2f} GB")
    print()
    print("| net | layer | op | N,H,W,Ci,Co,k,s | alg MB | read MB | write MB | measured / alg | excess MB |")
    print("|---|---|---|---|---|---|---|---|---|")
    rows = sorted(per_layer.items(), key=lambda kv: -(kv[1][2] + kv[1][3] - kv[1][1]))
    for (net, layer, op, shp), (n, alg, rd, w) in rows:
        print(f"| {net} | {layer} | {op} | {','.join(map(str, shp))} | {alg / 1e6:.0f} | {rd / 1e6:.0f} | "
              f"{w / 1e6:.0f} | {(rd + w) / max(alg, 1):.2f} | {(rd + w - alg) / 1e6:.0f} |")
    print()
    print("| other kernel | read MB | write MB |")
    print("|---|---|---|")
    for k, (rd, w) in sorted(other.items(), key=lambda kv: -(kv[1][0] + kv[1][1]))[:40]:
        print(f"| `{k}` | {rd / 1e6:.0f} | {w / 1e6:.0f} |")


def kernels(a):
    """Per conv call of the marked step: its dispatches (kernel, microseconds) from a
    rocprofv3 --kernel-trace CSV of `run` -- where the time of each layer op goes (GEMM, split
    passes, split-K reduce)."""
    meta = json.load(open(a.marks))
    marks, recs = meta["marks"], meta["records"]
    path = a.trace
    if os.path.isdir(path):
        found = [os.path.join(r, f) for r, _, fs in os.walk(path) for f in fs if f.endswith("kernel_trace.csv")]
        if len(found) != 1:
            raise SystemExit(f"{path}: {len(found)} kernel_trace.csv files")
        path = found[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"],
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows.sort()
    mi = [i for i, (_, k, _) in enumerate(rows) if "k_mark" in k]
    mi = mi[-len(marks):]
    calls = defaultdict(list)
    cur = None
    for j in range(len(mi) - 1):
        kind = marks[j]
        if isinstance(kind, list) and kind[0] == "begin":
            cur = kind[1]
        elif isinstance(kind, list) and kind[0] == "end":
            cur = None
        elif kind == "step_end":
            break
        if cur is None:
            continue
        for i in range(mi[j] + 1, mi[j + 1]):
            calls[cur].append((_short(rows[i][1]), rows[i][2]))
    sel = [s for s in (a.select or "").split(",") if s]
    for i, r in enumerate(recs):
        lab = f"{r['label']} {r['op']} {','.join(map(str, r['shape']))}"
        if sel and not any(s in lab for s in sel):
            continue
        ks = calls.get(i, [])
        print(f"{lab}: {sum(t for _, t in ks):.1f} us = " + " + ".join(f"{k} {t:.1f}" for k, t in ks))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="mode", required=True)
    r = sub.add_parser("run")
    r.add_argument("--model", default="pix2pix")
    r.add_argument("--batch", type=int, default=None)
    r.add_argument("--fp16", type=int, default=None)
    r.add_argument("--no-content", action="store_true")
    r.add_argument("--out", required=True)
    t = sub.add_parser("table")
    t.add_argument("--fetch", required=True)
    t.add_argument("--write", required=True)
    t.add_argument("--marks", required=True)
    k = sub.add_parser("kernels")
    k.add_argument("--trace", required=True)
    k.add_argument("--marks", required=True)
    k.add_argument("--select", default="", help="comma-separated substrings of 'label op shape' to print")
    a = ap.parse_args()
    {"run": run, "table": table, "kernels": kernels}[a.mode](a)


if __name__ == "__main__":
    main()
