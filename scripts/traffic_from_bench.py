#!/usr/bin/env python3
"""Write profiles/pmc_traffic*.json (the committed fallback of bench.py's roofline.traffic)
from bench lines whose traffic was measured live (two rocprofv3 --pmc child runs of the same
workload, bench.py pmc_leg), stamped with this tree's csrc_sha and the commit.

    python scripts/traffic_from_bench.py LABEL COMMIT gpurun_out/<tag>_bench*.json
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
from pmc_traffic import METHOD, csrc_sha  # noqa: E402

OUT = {"pix2pix": "pmc_traffic.json", "srgan": "pmc_traffic_srgan.json", "fsrgan": "pmc_traffic_fsrgan.json",
       "autoencoder": "pmc_traffic_autoencoder.json"}


def main(label, commit, paths):
    for p in paths:
        d = json.loads(open(p).read().strip().splitlines()[-1])
        r = d["roofline"]
        src = r.get("traffic_source") or ""
        if not r.get("traffic") or not src.startswith("live") or csrc_sha() not in src:
            raise SystemExit(f"{p}: traffic not measured live on this tree ({src[:80]})")
        metric = d["metric"]
        model = next(m for m in OUT if m in metric.lower() or (m == "fsrgan" and "fastsrgan" in metric.lower()))
        if model == "srgan" and "fastsrgan" in metric.lower():
            model = "fsrgan"
        t = {"conv_engine_bytes_per_step": r["traffic"], "steps": 3, "method": METHOD, "csrc_sha": csrc_sha(),
             "profile": label, "commit": commit, "workload": metric, "bench_value": d["value"]}
        with open(os.path.join(REPO, "profiles", OUT[model]), "w") as f:
            json.dump(t, f, indent=1)
        print(model, OUT[model], round(r["traffic"] / 1e9, 2), "GB/step")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
