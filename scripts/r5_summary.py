#!/usr/bin/env python3
"""Round-end numbers for DESIGN.md from one measurement set (scripts/gpu_r5_final.sh TAG):
the deep U-Net chain and narrow-layer times from the per-layer table, BN time and launches per
step from the rocprofv3 kernel stats (steps counted by the iteration-counter launches), launches per step.

    python scripts/r5_summary.py gpurun_out/r5_final"""
import csv
import sys

DEEP = {("G", n) for n in ("down6", "down7", "down8", "up1 (T)", "up2 (T)", "up3 (T)")}
NARROW = {("D", "down1"), ("D", "down1.g"), ("D", "last"), ("G", "down1"), ("G", "last (T)"),
          ("vgg19", "block1_conv1")}


def layers(path):
    rows = []
    for line in open(path):
        c = [x.strip() for x in line.strip().strip("|").split("|")]
        if len(c) < 16 or c[0] in ("net", "---"):
            continue
        rows.append(dict(net=c[0], layer=c[1], op=c[2], ms=float(c[11]), roof=float(c[15])))
    return rows


def stats(path, per_step):
    rows = list(csv.DictReader(open(path)))
    # (steps: the iteration-counter launches, one per network per step -- Adam may be split)
    steps = sum(int(r["Calls"]) for r in rows if "k_counter_add" in r["Name"]) / per_step
    tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e6 / steps
    bn = [r for r in rows if "k_bn_" in r["Name"]]
    bn_ms = sum(float(r["TotalDurationNs"]) for r in bn) / 1e6 / steps
    bn_n = sum(int(r["Calls"]) for r in bn) / steps
    launches = sum(int(r["Calls"]) for r in rows) / steps
    return steps, tot, bn_ms, bn_n, launches


def main(tag):
    L = layers(f"{tag}_layers_full.md")
    deep = [r for r in L if (r["net"], r["layer"]) in DEEP]
    nar = [r for r in L if (r["net"], r["layer"]) in NARROW]
    print(f"deep chain: {len(deep)} ops, {sum(r['ms'] for r in deep):.3f} ms/step, roof fractions "
          f"{min(r['roof'] for r in deep):.3f}-{max(r['roof'] for r in deep):.3f}")
    print(f"narrow layers: {len(nar)} ops, {sum(r['ms'] for r in nar):.3f} ms/step, roof fractions "
          f"{min(r['roof'] for r in nar):.3f}-{max(r['roof'] for r in nar):.3f}")
    for name, path, ad in (("pix2pix (streams)", f"{tag}_prof/run_kernel_stats.csv", 2),
                           ("pix2pix (one stream)", f"{tag}_prof_seq/run_kernel_stats.csv", 2),
                           ("srgan", f"{tag}_prof_srgan/run_kernel_stats.csv", 2),
                           ("fsrgan", f"{tag}_prof_fsrgan/run_kernel_stats.csv", 2)):
        try:
            s, tot, bn, bnn, n = stats(path, ad)
        except (OSError, ZeroDivisionError):
            continue
        print(f"{name}: {s:.0f} steps, kernels {tot:.2f} ms/step in {n:.0f} launches; BN {bn:.3f} ms in {bnn:.0f}")


if __name__ == "__main__":
    main(sys.argv[1])
