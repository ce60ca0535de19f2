"""fp16x3 generic-kernel check per forced tile config / split count (diagnostic):
python scripts/diag/x3_cfg_check.py -> max rel L2 error vs fp64 per (op, cfg)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r"""
import sys, torch
sys.path[:0] = [sys.argv[1] + '/denoise-gan_amd', sys.argv[1] + '/tests']
from dgan.ops import ConvDesc
from torch_ref import conv2d_ref, conv2d_transpose_ref
N, H, W, ci, co, tr = map(int, sys.argv[2:8])
torch.manual_seed(0)
d = ConvDesc(N, H, W, ci, co, 4, 2, 'same', bool(tr), math='f16x3')
x = torch.randn(N, H, W, ci, dtype=torch.float64); w = torch.randn(*d.weight_shape, dtype=torch.float64) * 0.05
dy = torch.randn(N, d.Ho, d.Wo, co, dtype=torch.float64)
xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
yr = conv2d_transpose_ref(xr, wr, 2, d.pads, (d.Ho, d.Wo), None) if tr else conv2d_ref(xr, wr, 2, d.pads, None)
yr.backward(dy)
xg, wg, dyg = x.float().cuda(), w.float().cuda(), dy.float().cuda()
y = torch.empty(d.out_shape, device='cuda'); d.fwd(xg, wg, y)
dx = torch.empty_like(xg); d.bwd_data(dyg, wg, dx)
dw = torch.empty_like(wg); d.bwd_filter(xg, dyg, dw)
torch.cuda.synchronize()
r = lambda a, b: float((a.double().cpu() - b).norm() / b.norm())
print(f"fwd {r(y, yr.detach()):.2e} bwd_data {r(dx, xr.grad):.2e} bwd_filter {r(dw, wr.grad):.2e}")
"""
for shape in (["4", "2", "2", "1024", "512", "1"], ["4", "4", "4", "512", "512", "0"], ["2", "16", "16", "256", "64", "1"]):
    for cfg in [None] + [str(c) for c in range(7)]:
        env = dict(os.environ, DG_PLAN_DEBUG="1")
        if cfg is not None:
            env["DG_FORCE_X3CFG"] = cfg
        r = subprocess.run([sys.executable, "-c", CHILD, REPO] + shape, env=env, capture_output=True, text=True,
                           timeout=120)
        plans = [l.split("->")[1].strip() for l in r.stderr.splitlines() if "[dg plan]" in l][-3:]
        out = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr.strip().splitlines()[-1][:200]
        print(" ".join(shape), "cfg", cfg, "|", out, "|", "; ".join(plans), flush=True)
