#!/usr/bin/env python3
"""Throughput of the pix2pix training step on MI355X (BASELINE.json metric:
training images/sec, pix2pix 256x256 bs16 per GPU, 1/2/4/8 GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One step = the reference's train_step (train_pix2pix.py:33-71) on 16 synthetic
256x256 noisy/clean pairs per GPU already resident in HBM: G(x), the identity
pass G(y), D real + fake, L1/L2/TV/GAN/identity losses, both gradients, the
data-parallel gradient all-reduce (N>1) and Keras-Adam on G and D, plus the
VGG19 content loss (pix2pix.py:45-51: VGG19-to-block5_conv4 forward on G(x)
and on y, backward into G(x)) with seeded stand-in weights (ImageNet weights
are a download; same FLOPs and shapes).  `--no-content` drops the VGG term;
at N=1 the same run also reports that content-free step as `core`.  fp32 tensors
throughout; the conv GEMMs use the library's default conv math, bf16x6
(fp32 operands split exactly into three bf16 pieces, the six significant
piece products accumulated in fp32 -- fp32-accurate); set
DG_CONV_MATH=fp32 for the exact-fp32 MFMA path.

Prints ONE JSON line (rank 0).  Extra fields:
  roofline      conv engine (the dominant kernels): algorithmic conv FLOPs of
                one step / summed conv launch time measured with HIP events on
                the launching stream, vs the peak of the conv math in use
                (bf16x6: bf16 dense peak / 6 = 419.4 TF/s; fp32: 157.3 TF/s)
  cpu_baseline  the CPU restatement of the same graph (oracle/torch_p2p.py,
                torch fp32 autograd) timed on this box's host cores, rank 0,
                N=1 only, bounded sample
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "denoise-gan_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_MFMA_PEAK = 157.3e12   # gfx950 dense fp32 MFMA (MI355X_MICROARCH.md)
BF16_MFMA_PEAK = 2516.6e12  # gfx950 dense bf16 MFMA: 1024 FLOP/clk/SIMD x 1024 SIMDs x 2.4 GHz
# bf16x6 conv math: six bf16 piece products per fp32 product, so its
# fp32-equivalent ceiling is the bf16 peak / 6
X6_PEAK = BF16_MFMA_PEAK / 6.0


class Args:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def synthetic_batch(n, size, seed):
    from dataloader import synthetic_pair
    return synthetic_pair(n, size, seed)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU")
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a captured HIP graph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-identity", action="store_true")
    ap.add_argument("--no-content", action="store_true", help="drop the VGG19 content term")
    ap.add_argument("--no-core", action="store_true", help="skip the content-free secondary measurement")
    ap.add_argument("--profile-only", action="store_true", help="skip roofline/cpu legs (for rocprofv3 runs)")
    ap.add_argument("--dist", action="store_true",
                    help="data-parallel path (process group + gradient all-reduce) even at world size 1")
    args = ap.parse_args()
    # the one JSON line goes to the original stdout; everything else written to
    # fd 1 (RCCL's version banner, library logs) is sent to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DG_DIST_BACKEND", "nccl") != "nccl":
        local %= max(1, torch.cuda.device_count())  # rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or args.dist
    if distributed:
        import torch.distributed as dist
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        backend = os.environ.get("DG_DIST_BACKEND", "nccl")  # gloo: rehearse N ranks on one GPU
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    import dgan
    dgan.build()  # no-op when the in-tree library is current
    from pix2pix import Pix2Pix
    from dgan import ops

    def build(content):
        m = Pix2Pix(Args(crop_size=args.size, retrain=0, width=1, seed=1234, dropout_seed=rank,
                         identity_loss=0 if args.no_identity else 1, content_loss=int(content)))
        if distributed:
            from dgan.dist import setup_data_parallel
            setup_data_parallel(m)
        return m

    x_np, y_np = synthetic_batch(args.batch, args.size, seed=1000 + rank)
    x = torch.from_numpy(x_np).to(dev)
    y = torch.from_numpy(y_np).to(dev)
    # N=1: the step is captured once into a HIP graph and replayed (eager
    # launches if capture fails).  N>1 launches eagerly: measured at N=1, eager
    # runs at the graph's rate (598.7 vs 599.0 img/s), so no rank needs to rely
    # on multi-rank RCCL graph capture (a world-size-1 RCCL group does capture)
    use_graph = not args.no_graph and world == 1

    def measure(content):
        model = build(content)
        trainer = model.trainer(x.shape)
        for _ in range(max(1, args.warmup // 2)):
            trainer.step(x, y)
        torch.cuda.synchronize()
        graph = None
        if use_graph:
            try:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    trainer.step(x, y)
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    trainer.step(x, y)
                torch.cuda.synchronize()
            except Exception as e:  # report, fall back to eager launches
                print(f"[bench] graph capture failed ({e}); eager launches", file=sys.stderr)
                graph = None

        def step():
            if graph is not None:
                graph.replay()
            else:
                trainer.step(x, y)

        for _ in range(args.warmup - max(1, args.warmup // 2)):
            step()
        torch.cuda.synchronize()
        # ---- timed region: barrier + sync on both sides, max over ranks ----
        if distributed:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if distributed:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if distributed:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return model, trainer, graph, elapsed

    content = not args.no_content
    model, trainer, graph, elapsed = measure(content)
    hip_graph = graph is not None
    conv_math = "bf16x6" if trainer.G.ldesc.math == ops.MATH_BF16X6 else "fp32"
    losses = trainer.loss.cpu().numpy()
    ms_per_step = elapsed / args.steps * 1e3
    images = world * args.batch * args.steps
    value = images / elapsed

    # ---- roofline of the conv engine (HIP events, eager pass) ---------------
    roofline = None
    step_flops = None
    if not args.profile_only:
        with ops.ConvProfile() as prof:
            trainer.step(x, y)
        torch.cuda.synchronize()
        recs = prof.summary()
        conv_flops = sum(r["flops"] for r in recs)
        conv_alg_bytes = sum(r["bytes"] for r in recs)
        conv_ms = sum(r["ms"] for r in recs)
        step_flops = conv_flops
        achieved = conv_flops / (conv_ms * 1e-3)
        peak = X6_PEAK if conv_math == "bf16x6" else FP32_MFMA_PEAK
        traffic = None
        tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(tpath) and content:
            with open(tpath) as f:
                traffic = round(json.load(f)["conv_engine_bytes_per_step"], 0)
        roofline = {"bound": "mfma", "achieved": round(achieved / 1e12, 2), "peak": round(peak / 1e12, 1),
                    "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                    "traffic_unit": "HBM bytes per step over the conv-engine launches (rocprofv3 PMC, "
                                    "profiles/pmc_traffic.json; algorithmic operand bytes per step: "
                                    f"{round(conv_alg_bytes / 1e9, 2)} GB)",
                    "kernel": "dg conv engine (k_conv_gemm_x6 / k_conv_gemm + split passes + narrow + split-K "
                              "reduce), all conv launches of one step",
                    "peak_basis": ("bf16 dense MFMA peak / 6 (six bf16 piece products per fp32 product)"
                                   if conv_math == "bf16x6" else "fp32 dense MFMA peak"),
                    "frac_of_fp32_mfma_peak": round(achieved / FP32_MFMA_PEAK, 4),
                    "conv_launch_ms_per_step": round(conv_ms, 3), "conv_gflop_per_step": round(conv_flops / 1e9, 1),
                    "step_frac": round(conv_flops / (ms_per_step * 1e-3) / peak, 4)}
        if rank == 0 and os.environ.get("DG_BENCH_DETAIL"):
            for r in sorted(recs, key=lambda r: -r["ms"])[:int(os.environ.get("DG_BENCH_DETAIL_N", "60"))]:
                print(json.dumps({**r, "tflops": r["flops"] / (r["ms"] * 1e-3) / 1e12}), file=sys.stderr)

    core = None
    if content and world == 1 and not args.no_core and not args.profile_only:
        _, _, _, el_core = measure(False)
        core = {"value": round(images / el_core, 2), "ms_per_step": round(el_core / args.steps * 1e3, 3),
                "workload": "the same step without the VGG19 content term (pix2pix.py:87 weight 0)"}

    # ---- CPU baseline: torch fp32 restatement, rank 0, N=1 only -------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_only:
        cpu = cpu_baseline(args.size, args.cpu_seconds, identity=not args.no_identity,
                           vgg=model.vgg.arena.export() if model.vgg is not None else None)

    if rank == 0:
        out = {
            "metric": "training images/sec, pix2pix 256x256 bs16/GPU",
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "conv_math": conv_math,
            "data": "synthetic (seeded noisy/clean 256x256 pairs resident in HBM; random-init weights)",
            "config": {"workload": "pix2pix train_step (train_pix2pix.py:33-71): G(x)+G(y) identity pass, D real+fake, "
                                   "GAN/L1/L2/TV/identity losses, D and G gradients, Keras Adam G and D; "
                                   + ("VGG19 content loss (seeded stand-in weights: ImageNet weights are a download)"
                                      if content else "VGG content term 0"),
                       "model": "pix2pix U-Net G (54.4M) + PatchGAN D (2.77M)",
                       "global_batch": world * args.batch, "batch_per_gpu": args.batch, "image_size": args.size,
                       "parallelism": f"dp{world}", "hip_graph": hip_graph,
                       "identity_pass": not args.no_identity,
                       "conv_gflop_per_image": round(step_flops / args.batch / 1e9, 2) if step_flops else None},
            "losses": [round(float(v), 6) for v in losses],
            "core": core,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), file=json_out, flush=True)
    if distributed:
        dist.destroy_process_group()


def cpu_baseline(size, seconds, identity=True, vgg=None):
    """The oracle's torch-fp32 restatement of the same step on the host cores."""
    from oracle import torch_p2p as T
    from oracle import p2p_oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    torch.set_num_threads(threads)
    bs = 2
    G = O.init_variables(O.g_variables(1), 1234)
    D = O.init_variables(O.d_variables(1), 1235)
    step = T.make_fp32_step(G, D, PV=vgg)
    x, y = O.synthetic_pair(bs, size, seed=7)
    step(x, y)  # warm-up
    n = 0
    t0 = time.perf_counter()
    while True:
        step(x, y)
        n += 1
        if time.perf_counter() - t0 > seconds or n >= 20:
            break
    el = time.perf_counter() - t0
    return {"value": round(n * bs / el, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} steps x {bs} images at {size}x{size}, torch fp32 CPU autograd restatement "
                      f"(oracle/torch_p2p.py) incl. identity pass, {'VGG19 content loss, ' if vgg else ''}"
                      f"Keras-Adam; {el:.1f}s"}


if __name__ == "__main__":
    main()
