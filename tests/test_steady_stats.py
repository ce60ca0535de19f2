"""scripts/steady_stats.py: per-step kernel statistics over the last complete steps of a
rocprofv3 kernel trace (steps delimited by the two iteration-counter launches per step), so
warm-up and one-time launches stay out of the per-step numbers."""
import csv
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path):
    rows, t = [], 0

    def k(name, dur):
        nonlocal t
        rows.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + dur})
        t += dur + 10

    k("warmup_only_kernel", 5000)   # one-time work before the steps
    for _ in range(4):              # four steps: G counter, conv, bn, D counter
        k("dg::k_counter_add(int*)", 100)
        k("dg::k_conv_gemm_x6<...>", 2000)
        k("dg::k_bn_apply<4>", 300)
        k("dg::k_counter_add(int*)", 100)
    k("dg::k_counter_add(int*)", 100)   # the next step's first mark
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)


def test_steady_stats_counts_only_complete_steps(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p)
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "steady_stats.py"), str(p), "3"],
                       capture_output=True, text=True, check=True)
    rows = {row["Name"]: row for row in csv.DictReader(line for line in r.stdout.splitlines())}
    assert "warmup_only_kernel" not in rows
    assert float(rows["dg::k_conv_gemm_x6<...>"]["CallsPerStep"]) == 1.0
    assert float(rows["dg::k_conv_gemm_x6<...>"]["UsPerStep"]) == 2.0
    assert float(rows["dg::k_counter_add(int*)"]["CallsPerStep"]) == 2.0
    assert "3 steady steps" in r.stderr
