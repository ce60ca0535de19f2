#!/usr/bin/env python3
"""Achievable dense bf16 MFMA rate on this MI355X: the vendor GEMM (torch.matmul
-> hipBLASLt) on uniform random [-1, 1) bf16 operands, square sizes, HIP-event
median of repeats, as a fraction of the nominal 2516.6 TF/s dense peak.  The
bf16x6 conv kernels run six bf16 products per fp32 product, so their
fp32-equivalent rate divided by (this rate / 6) is their fraction of what the
matrix cores deliver at the clock the chip holds under a dense bf16 load
(MI355X_MICROARCH.md 'DVFS give-back', cdna_hip_programming.md §5.4 rule 25)."""
import torch

PEAK = 2516.6e12


def main():
    torch.manual_seed(0)
    for n in (4096, 8192):
        a = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
        for _ in range(5):
            torch.matmul(a, b)
        ts = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            torch.matmul(a, b)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = sorted(ts)[len(ts) // 2]
        tf = 2.0 * n ** 3 / (ms * 1e-3)
        print(f"bf16 GEMM {n}^3 (hipBLASLt, random [-1,1)): {ms:.3f} ms = {tf / 1e12:.1f} TF/s = {tf / PEAK:.3f} of "
              f"the nominal dense peak; bf16x6 equivalent {tf / 6e12:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
