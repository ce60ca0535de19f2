#!/usr/bin/env python3
"""Throughput of the GAN training steps on MI355X (BASELINE.json metric:
training images/sec, pix2pix 256x256 bs16 per GPU, 1/2/4/8 GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model pix2pix|srgan|fsrgan|autoencoder]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Workloads (one "step" = the reference's train_step on one synthetic batch
already resident in HBM, per GPU):
  pix2pix      (default, the headline) train_pix2pix.py:33-71 at 256x256, 16
               noisy/clean pairs: G(x), the identity pass G(y), D real +
               fake, L1/L2/TV/GAN/identity losses, the VGG19 content loss
               (pix2pix.py:45-51; seeded stand-in weights, ImageNet weights
               are a download; same FLOPs and shapes), both gradients, the
               data-parallel all-reduce (N>1), Keras-Adam on G and D.
               `--no-content` drops the VGG term; at N=1 that content-free
               step is also reported as `core` (the north star's
               "L1 + adversarial" step).                     BASELINE configs[1]
  srgan        train_srgan.py:61-118, 4x SR 24 -> 96, 16 residual blocks,
               bs32, VGG19 content loss                     BASELINE configs[2]
  fsrgan       train_fsrgan.py:61-120, 128 -> 512, bs8 per GPU
                                                            BASELINE configs[4]
  autoencoder  train_autoencoder.py:66-112, 64x64 grayscale (replicated to
               3 channels), bs4                             BASELINE configs[0]
fp32 tensors throughout; the conv GEMMs use the library's default conv
math, bf16x6 (fp32 operands split exactly into three bf16 pieces, the six
significant piece products accumulated in fp32 -- fp32-accurate, see
DESIGN.md); DG_CONV_MATH=fp32 selects the exact-fp32 MFMA path.

Prints ONE JSON line (rank 0).  Extra fields:
  roofline      conv engine (the dominant kernels): algorithmic conv FLOPs of
                one step / summed conv launch time measured with HIP events on
                the launching stream, vs the peak of the conv math in use
                (bf16x6: bf16 dense peak / 6 = 419.4 TF/s; fp32: 157.3 TF/s);
                `traffic` = HBM bytes per step of those launches, measured
                live: two rocprofv3 --pmc child runs (FETCH_SIZE, WRITE_SIZE)
                of the same workload (N=1, rank 0; --no-pmc-leg falls back to
                the committed profile when its csrc_sha matches this tree)
  cpu_baseline  the CPU restatement of the same step (oracle/, torch fp32
                autograd) timed on this box's host cores, rank 0, N=1 only,
                bounded sample of the same workload
"""
import argparse
import contextlib
import json
import os
import subprocess
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
# fp16x3 conv math: three fp16 piece products (fp16 MFMA rate = bf16) per fp32 product
X3_PEAK = BF16_MFMA_PEAK / 3.0
ARITH_PEAK = {"fp32": FP32_MFMA_PEAK, "bf16x6": X6_PEAK, "fp16": BF16_MFMA_PEAK, "f16x3": X3_PEAK}

WORKLOADS = {
    "pix2pix": dict(metric="training images/sec, pix2pix 256x256 bs16/GPU", batch=16, size=256, scale=1,
                    model="pix2pix U-Net G (54.4M) + PatchGAN D (2.77M)", traffic="pmc_traffic.json"),
    "srgan": dict(metric="training images/sec, SRGAN 4x 24->96 bs32/GPU", batch=32, size=96, scale=4,
                  model="SRGAN G (16 residual blocks) + SR D", traffic="pmc_traffic_srgan.json",
                  fp16=1),   # train_srgan.py:275 defaults to the mixed_float16 policy
    "fsrgan": dict(metric="training images/sec, FastSRGAN 4x 128->512 bs8/GPU", batch=8, size=512, scale=4,
                   model="FastSRGAN G (6 inverted-residual blocks) + SR D", traffic="pmc_traffic_fsrgan.json",
                   cpu_batch=1),   # CPU sample: one 512x512 image per step (~20 s per step on 16 cores)
    "autoencoder": dict(metric="training images/sec, autoencoder 64x64 grayscale bs4/GPU", batch=4, size=64,
                        scale=1, model="conv autoencoder G + sigmoid D", traffic="pmc_traffic_autoencoder.json",
                        gray=True),
}


class Args:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def synthetic_batch(wl, n, seed):
    from dataloader import synthetic_pair
    x, y = synthetic_pair(n, wl["size"], seed)
    if wl.get("gray"):
        x = np.repeat(x.mean(-1, keepdims=True), 3, -1).astype(np.float32)
        y = np.repeat(y.mean(-1, keepdims=True), 3, -1).astype(np.float32)
    if wl["scale"] > 1:
        x = np.ascontiguousarray(x[:, ::wl["scale"], ::wl["scale"]])
    return x, y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="pix2pix", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default: the workload's)")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of a captured HIP graph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=3, help="CPU baseline: timed steps at the full batch")
    ap.add_argument("--no-identity", action="store_true")
    ap.add_argument("--no-content", action="store_true", help="drop the VGG19 content term")
    ap.add_argument("--no-core", action="store_true", help="skip the content-free secondary measurement")
    ap.add_argument("--profile-only", action="store_true", help="skip roofline/cpu legs (for rocprofv3 runs)")
    ap.add_argument("--no-pmc-leg", action="store_true",
                    help="do not measure roofline.traffic live (two rocprofv3 --pmc child runs, FETCH_SIZE and "
                         "WRITE_SIZE, N=1 rank 0 only); use the committed profile if it matches the sources")
    ap.add_argument("--fp16", type=int, default=None,
                    help="SR family: mixed_float16 (fp16 conv GEMMs + dynamic loss scale); default: the "
                         "reference driver's (train_srgan.py fp16=1, the others 0)")
    ap.add_argument("--dist", action="store_true",
                    help="data-parallel path (process group + gradient all-reduce) even at world size 1")
    ap.add_argument("--no-twin", action="store_true",
                    help="pix2pix: skip the bf16x6 twin measurement (fp32_exact: every conv GEMM on six bf16 "
                         "piece products instead of fp16x3)")
    args = ap.parse_args()
    wl = WORKLOADS[args.model]
    batch = args.batch or wl["batch"]
    fp16 = bool(wl.get("fp16", 0) if args.fp16 is None else args.fp16) and args.model != "pix2pix"
    # the one JSON line goes to the original stdout; everything else written to
    # fd 1 (RCCL's version banner, library logs) is sent to stderr
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(f"bench.py --gpus {args.gpus}: launch one process per GPU with "
                 f"`python -m torch.distributed.run --nproc-per-node {args.gpus} ... bench.py --gpus {args.gpus}`")
    if "WORLD_SIZE" in os.environ and world != args.gpus:
        sys.exit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world} (torch.distributed.run --nproc-per-node "
                 f"must equal --gpus)")
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
        # no fallback: a process group that cannot be built on RCCL ends the run
        if backend == "nccl":
            if not dist.is_nccl_available():
                sys.exit("bench.py: torch.distributed has no nccl (RCCL) backend in this build")
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        if dist.get_backend() != backend or dist.get_world_size() != world:
            sys.exit(f"bench.py: process group is {dist.get_backend()} x{dist.get_world_size()}, "
                     f"expected {backend} x{world}")

    import dgan
    dgan.build()  # no-op when the in-tree library is current
    from dgan import ops

    def build(content):
        if args.model == "pix2pix":
            from pix2pix import Pix2Pix
            m = Pix2Pix(Args(crop_size=wl["size"], retrain=0, width=1, seed=1234, dropout_seed=rank,
                             identity_loss=0 if args.no_identity else 1, content_loss=int(content)))
        else:
            from autoencoder import Autoencoder
            from fsrgan import FastSRGAN
            from srgan import SRGAN
            cls = {"srgan": SRGAN, "fsrgan": FastSRGAN, "autoencoder": Autoencoder}[args.model]
            m = cls(Args(crop_size=wl["size"], scale=wl["scale"], lr=1e-3, fp16=int(fp16), retrain=0, seed=1234,
                         content_loss=int(content)))
        if distributed:
            from dgan.dist import setup_data_parallel
            setup_data_parallel(m)
        return m

    x_np, y_np = synthetic_batch(wl, batch, seed=1000 + rank)
    x = torch.from_numpy(x_np).to(dev)
    y = torch.from_numpy(y_np).to(dev)
    # The step is captured once into a HIP graph and replayed, at every N: with the five-stream
    # step of round 5 eager launches lost 3.7 % at world 1 through RCCL (939 / 941 vs 974 / 977
    # img/s, profiles/r6/dist_graph_eager.txt).  The captured all-reduces go to a capture-only
    # process group (dgan.dist.capture_group).  Every rank must take the same path: the ranks
    # agree on the capture's success (an all-reduce MIN on the default group) and all fall back
    # to eager launches if any rank's capture failed.  (A gloo rehearsal, DG_DIST_BACKEND=gloo, has
    # no capturable collectives: eager at N>1.)
    use_graph = not args.no_graph and (world == 1 or os.environ.get("DG_DIST_BACKEND", "nccl") == "nccl")

    def trainer_of(model):
        return model.trainer(x.shape) if args.model == "pix2pix" else model.trainer(x.shape, y.shape)

    def measure(content, twin=False):
        if twin:   # every pix2pix / VGG19 GEMM in bf16x6 (fp32-accurate operands) instead of fp16x3
            from dgan import nets as _nets_t
            saved = (_nets_t.P2P_MATH, os.environ.get("DG_VGG_MATH"))
            _nets_t.P2P_MATH = "bf16x6"
            os.environ["DG_VGG_MATH"] = "bf16x6"
            try:
                return measure(content)
            finally:
                _nets_t.P2P_MATH = saved[0]
                if saved[1] is None:
                    os.environ.pop("DG_VGG_MATH", None)
                else:
                    os.environ["DG_VGG_MATH"] = saved[1]
        model = build(content)
        trainer = trainer_of(model)
        for _ in range(max(1, args.warmup // 2)):
            trainer.step(x, y)
        torch.cuda.synchronize()
        graph = None
        if use_graph:
            from dgan.dist import CAPTURE_MODE
            try:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    trainer.step(x, y)
                torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                graph = torch.cuda.CUDAGraph()
                # (collectives inside the capture go to a capture-only process group, dist.capture_group;
                # thread-local capture mode leaves the watchdog threads free to query eager events)
                with (model.grad_sync.capturing() if distributed else contextlib.nullcontext()):
                    with torch.cuda.graph(graph, capture_error_mode=CAPTURE_MODE):
                        trainer.step(x, y)
                torch.cuda.synchronize()
            except Exception as e:  # report, fall back to eager launches
                print(f"[bench] graph capture failed ({e}); eager launches", file=sys.stderr)
                graph = None
            if distributed and world > 1:
                ok = torch.tensor([1 if graph is not None else 0], dtype=torch.int32, device=dev)
                dist.all_reduce(ok, op=dist.ReduceOp.MIN)
                if int(ok.item()) == 0 and graph is not None:
                    print("[bench] another rank's capture failed; eager launches on every rank", file=sys.stderr)
                    graph = None
        check = None
        # (--profile-only: the check's snapshot copies and comparisons would land in the profiled
        # window as non-step kernels -- at::native compares, rocclr copies -- so it runs only in
        # the measured bench)
        if graph is not None and not args.profile_only:
            check = graph_vs_eager(trainer, graph, x, y, strict=world == 1)

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
        measure.check = check
        return model, trainer, graph, elapsed

    content = not args.no_content
    model, trainer, graph, elapsed = measure(content)
    graph_check = measure.check
    hip_graph = graph is not None
    conv_math = "fp16" if fp16 else ("bf16x6" if ops.default_conv_math() == ops.MATH_BF16X6 else "fp32")
    if not fp16 and args.model != "pix2pix" and content:
        from dgan.sr_trainer import VGGNetwork
        if wl["size"] ** 2 >= VGGNetwork.X3_MIN_PIXELS and not os.environ.get("DG_VGG_MATH"):
            conv_math = f"G/D {conv_math}, VGG19 f16x3"
    if args.model == "pix2pix":
        from dgan import nets as _nets
        conv_math = f"G/D {_nets.P2P_MATH}, VGG19 {os.environ.get('DG_VGG_MATH', 'f16x3')}"
    losses = trainer.loss.cpu().numpy()
    ms_per_step = elapsed / args.steps * 1e3
    images = world * batch * args.steps
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
        # each op against the dense MFMA peak of the arithmetic its GEMM runs in (ops.op_arith):
        # peak = total FLOPs / the time they take at those peaks, frac = that time / launch time
        t_peak = sum(r["flops"] / ARITH_PEAK[r["arith"]] for r in recs)
        peak = conv_flops / t_peak if t_peak > 0 else X6_PEAK
        arith_mix = {}
        for r in recs:
            arith_mix[r["arith"]] = arith_mix.get(r["arith"], 0.0) + r["flops"] / 1e9
        traffic, source = traffic_of(args, wl, content, batch, rank, world)
        roofline = {"bound": "mfma", "achieved": round(achieved / 1e12, 2), "peak": round(peak / 1e12, 1),
                    "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                    "traffic_unit": "HBM bytes per step over the conv-engine launches (rocprofv3 PMC "
                                    "FETCH_SIZE x2 + WRITE_SIZE); algorithmic fp32 operand bytes per step: "
                                    f"{round(conv_alg_bytes / 1e9, 2)} GB",
                    "traffic_source": source,
                    "kernel": "dg conv engine (k_conv_gemm_x6 / k_conv_gemm + split passes + narrow + split-K "
                              "reduce), all conv launches of one step",
                    "peak_basis": "per op, the dense MFMA peak of its GEMM's arithmetic: fp16x3 bf16-rate peak / 3 "
                                  "(three fp16 piece products per fp32 product), bf16x6 / 6, fp16 / 1, fp32 MFMA; "
                                  "peak = total FLOPs / their time at those peaks",
                    "gflop_by_arith": {k: round(v, 1) for k, v in sorted(arith_mix.items())},
                    "frac_of_bf16x6_basis": round(achieved / X6_PEAK, 4),
                    "frac_of_fp32_mfma_peak": round(achieved / FP32_MFMA_PEAK, 4),
                    "conv_launch_ms_per_step": round(conv_ms, 3), "conv_gflop_per_step": round(conv_flops / 1e9, 1),
                    "step_frac": round(conv_flops / (ms_per_step * 1e-3) / peak, 4)}
        # per network (conv descriptor labels "G.down1", "D.last", "vgg19.block1_conv1", ...);
        # for pix2pix, `p2p_convs` = the G + D Conv2D / Conv2DTranspose kernels the north star's
        # ">= 40 % of MFMA peak" names (pix2pix.py:110-142, 194-220), VGG19 excluded

        nets = {}
        for r in recs:
            net = (r["label"] or "?").split(".", 1)[0]
            a = nets.setdefault(net, [0.0, 0.0, 0.0])
            a[0] += r["flops"]
            a[1] += r["ms"]
            a[2] += r["flops"] / ARITH_PEAK[r["arith"]]

        def frac_of(fl, ms, tp):
            return {"gflop_per_step": round(fl / 1e9, 1), "ms_per_step": round(ms, 3),
                    "achieved": round(fl / (ms * 1e-3) / 1e12, 2), "frac": round(tp / (ms * 1e-3), 4),
                    "frac_of_bf16x6_basis": round(fl / (ms * 1e-3) / X6_PEAK, 4)}
        roofline["by_net"] = {n: frac_of(*v) for n, v in sorted(nets.items()) if v[1] > 0}
        if args.model == "pix2pix" and "G" in nets and "D" in nets:
            fl, ms = nets["G"][0] + nets["D"][0], nets["G"][1] + nets["D"][1]
            tp = nets["G"][2] + nets["D"][2]
            roofline["p2p_convs"] = {**frac_of(fl, ms, tp), "nets": "G + D (VGG19 excluded)",
                                     "target_frac": 0.40}
        if rank == 0 and os.environ.get("DG_BENCH_DETAIL"):
            for r in sorted(recs, key=lambda r: -r["ms"])[:int(os.environ.get("DG_BENCH_DETAIL_N", "60"))]:
                print(json.dumps({**r, "tflops": r["flops"] / (r["ms"] * 1e-3) / 1e12}), file=sys.stderr)

    core = None
    if args.model == "pix2pix" and content and world == 1 and not args.no_core and not args.profile_only:
        del model, trainer, graph
        torch.cuda.empty_cache()
        _, _, _, el_core = measure(False)
        core = {"value": round(images / el_core, 2), "ms_per_step": round(el_core / args.steps * 1e3, 3),
                "workload": "the same step without the VGG19 content term (pix2pix.py:87 weight 0)"}

    twin = None
    if (args.model == "pix2pix" and world == 1 and not args.no_twin and not args.profile_only
            and os.environ.get("DG_P2P_MATH", "f16x3") == "f16x3"):
        torch.cuda.empty_cache()
        _, _, _, el_twin = measure(content, twin=True)
        twin = {"value": round(images / el_twin, 2), "ms_per_step": round(el_twin / args.steps * 1e3, 3),
                "conv_math": "bf16x6 (G / D and VGG19: six bf16 piece products per fp32 product, dropped terms "
                             "< 2^-26)",
                "workload": "the same step (same flags) with every fp16x3 GEMM on bf16x6"}

    # ---- CPU baseline: torch fp32 restatement, rank 0, N=1 only -------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_only:
        cpu = cpu_baseline(args, wl, batch, content)

    if rank == 0:
        if args.model == "pix2pix":
            workload = ("pix2pix train_step (train_pix2pix.py:33-71): G(x)+G(y) identity pass, D real+fake, "
                        "GAN/L1/L2/TV/identity losses, D and G gradients, Keras Adam G and D; "
                        + ("VGG19 content loss (seeded stand-in weights: ImageNet weights are a download)"
                           if content else "VGG content term 0"))
        else:
            workload = (f"{args.model} train_step (train_{args.model}.py): G, D real+fake, VGG19 content loss "
                        f"(seeded stand-in weights), GAN/MAE/MSE/TV losses, both gradients, Adam with "
                        f"ExponentialDecay (D lr x5)"
                        + ("; mixed_float16: fp16 conv GEMMs, dynamic loss scale (LossScaleOptimizer)"
                           if fp16 else ""))
        out = {
            "metric": wl["metric"],
            "value": round(value, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": ("fp16 GEMM operands, fp32 accumulation (mixed_float16)" if fp16 else
                      "fp32 (GEMMs fp16x3, operands 2^-22)" if "f16x3" in conv_math else "fp32"),
            "conv_math": conv_math,
            "data": f"synthetic (seeded noisy/clean {wl['size']}x{wl['size']} pairs resident in HBM; "
                    "random-init weights)",
            "config": {"workload": workload, "model": wl["model"], "global_batch": world * batch,
                       "batch_per_gpu": batch, "image_size": wl["size"], "scale": wl["scale"],
                       "parallelism": f"dp{world}", "hip_graph": hip_graph,
                       "process_group": dist.get_backend() if distributed else None,
                       "identity_pass": not args.no_identity if args.model == "pix2pix" else None,
                       "conv_gflop_per_image": round(step_flops / batch / 1e9, 2) if step_flops else None},
            "lib": _lib_build_info(),
            "losses": [round(float(v), 6) for v in losses],
            "graph_equals_eager": graph_check,
            "core": core,
            "fp32_exact": twin,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), file=json_out, flush=True)
    if distributed:
        dist.destroy_process_group()


def graph_vs_eager(trainer, graph, x, y, strict=True):
    """The timed work is the tested work: from one snapshot of every tensor the step carries
    (both networks' parameters, gradients, Adam slots and counters, BN moving statistics, the
    losses), one eager step and one replay of the captured graph must end bit-identical.  The
    eager step is the launch sequence the -m gpu parity tests check against the fp64 oracle.
    strict (N=1): a difference ends the run; N>1: reported (the eager and the captured
    all-reduces run on two RCCL communicators).  The snapshot is restored afterwards."""
    from dgan.trainer import restore, snapshot, state_diff
    torch.cuda.synchronize()
    s0 = snapshot(trainer)
    trainer.step(x, y)
    eager = snapshot(trainer)
    restore(trainer, s0)
    graph.replay()
    replay = snapshot(trainer)
    torch.cuda.synchronize()
    bad = state_diff(eager, replay)
    restore(trainer, s0)
    torch.cuda.synchronize()
    if bad and strict:
        sys.exit(f"bench.py: the graph replay differs from the eager step in {bad[:8]} ({len(bad)} tensors)")
    if bad:
        print(f"[bench] graph replay != eager step in {len(bad)} tensors: {bad[:8]}", file=sys.stderr)
    return {"equal": not bad, "tensors": len(eager), "differing": bad[:8],
            "what": "one eager step and one graph replay from the same snapshot of parameters, gradients, Adam "
                    "slots, iteration counters, BN moving statistics and losses (G and D)"}


def _lib_build_info():
    """Provenance of the library this run loaded: the source hash compiled into it (dg_build_info)
    next to the hash of this tree's sources."""
    from dgan import _lib
    from dgan.build import LIB_PATH, source_sha
    info = _lib.build_info()
    return {"path": os.path.relpath(LIB_PATH, REPO), "built_from_source_sha": info.get("source_sha"),
            "tree_source_sha": source_sha(), "matches_tree": info.get("source_sha") == source_sha(),
            "hip": info.get("hip")}


def traffic_of(args, wl, content, batch, rank, world):
    """(HBM bytes per step of the conv engine, where the number came from)."""
    if not args.no_pmc_leg and rank == 0 and world == 1:
        try:
            return pmc_leg(args, batch)
        except Exception as e:  # report and fall back to the committed profile
            print(f"[bench] PMC leg failed ({e}); using the committed profile", file=sys.stderr)
    path = os.path.join(REPO, "profiles", wl["traffic"])
    default_fp16 = bool(wl.get("fp16", 0))
    if (not content or batch != wl["batch"] or args.no_identity or not os.path.exists(path)
            or (args.fp16 is not None and bool(args.fp16) != default_fp16)):
        return None, None   # the committed profile is of the default workload only
    with open(path) as f:
        t = json.load(f)
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    from pmc_traffic import csrc_sha
    if t.get("csrc_sha") != csrc_sha():   # measured on other kernels: not this tree's traffic
        return None, f"profiles/{wl['traffic']} was measured on other library sources; no live PMC leg"
    return (round(t["conv_engine_bytes_per_step"], 0),
            f"profiles/{wl['traffic']}: {t.get('profile', '?')} (commit {t.get('commit', '?')}, csrc_sha "
            f"{t['csrc_sha']} = this tree), {t.get('method', '')}")


def pmc_leg(args, batch):
    """Two rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE: they do not fit one
    pass) over a short --profile-only run of this same workload, as child processes."""
    import tempfile
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    from pmc_traffic import summarise
    steps = 3
    out = tempfile.mkdtemp(prefix="dg_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
    # the child measures THIS workload: every flag that changes the step is passed on
    child = [sys.executable, os.path.join(REPO, "bench.py"), "--profile-only", "--no-graph", "--steps", str(steps),
             "--warmup", "2", "--model", args.model, "--batch", str(batch)]
    if args.fp16 is not None:
        child += ["--fp16", str(int(args.fp16))]
    if args.no_content:
        child.append("--no-content")
    if args.no_identity:
        child.append("--no-identity")
    csvs = []
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out, ctr)
        subprocess.run(["timeout", "-s", "KILL", "300", "rocprofv3", "--pmc", ctr, "-d", d, "-o", "pmc",
                        "--output-format", "csv", "--"] + child, check=True, stdout=subprocess.DEVNULL,
                       stderr=subprocess.DEVNULL)
        found = [os.path.join(r, f) for r, _, fs in os.walk(d) for f in fs if f.endswith("counter_collection.csv")]
        if not found:
            raise RuntimeError(f"no counter_collection.csv for {ctr}")
        csvs.append(found[0])
    # the child runs warmup + timed steps + nothing else: count every launch, divide by the step count
    t = summarise(csvs[0], csvs[1], steps + 2)
    return (round(t["conv_engine_bytes_per_step"], 0),
            f"live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE child runs of this workload in this bench run, "
            f"csrc_sha {t['csrc_sha']} ({t['method']})")


def cpu_baseline(args, wl, batch, content):
    """The oracle's torch-fp32 restatement of the same step on the host cores, at the full batch."""
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    torch.set_num_threads(threads)
    if args.model == "pix2pix":
        from oracle import p2p_oracle as O
        from oracle import torch_p2p as T
        from dgan.graph import init_graph_variables
        from dgan.zoo import vgg19_features
        G = O.init_variables(O.g_variables(1), 1234)
        D = O.init_variables(O.d_variables(1), 1235)
        PV = init_graph_variables(vgg19_features(1), 1241) if content else None
        step = T.make_fp32_step(G, D, PV=PV)
        what = (f"torch fp32 CPU autograd restatement (oracle/torch_p2p.py) incl. identity pass, "
                f"{'VGG19 content loss, ' if content else ''}Keras-Adam")
    else:
        from oracle import sr_oracle as S
        from dgan import zoo
        from dgan.graph import init_graph_variables
        g = {"srgan": lambda: zoo.srgan_generator(scale=wl["scale"]), "fsrgan": zoo.fsrgan_generator,
             "autoencoder": zoo.autoencoder_generator}[args.model]()
        st = S.SRState(args.model, init_graph_variables(g, 1234), init_graph_variables(zoo.sr_discriminator(), 1235),
                       init_graph_variables(vgg19_features_(), 1241) if content else None, scale=wl["scale"],
                       dtype=np.float32)

        def step(x, y):
            S.train_step(st, x, y, apply=True)
        what = f"torch fp32 CPU autograd restatement (oracle/sr_oracle.py) incl. VGG19 content loss, Adam"
    cb = wl.get("cpu_batch", batch)
    x, y = synthetic_batch(wl, cb, seed=7)
    step(x, y)  # warm-up
    t0 = time.perf_counter()
    n = 0
    min_steps = args.cpu_steps if cb == batch else 1
    while n < min_steps or (time.perf_counter() - t0 < 10.0 and n < 200):   # >= min_steps and ~10 s
        step(x, y)
        n += 1
    el = time.perf_counter() - t0
    size = f"{wl['size'] // wl['scale']} -> {wl['size']}" if wl["scale"] > 1 else f"{wl['size']}x{wl['size']}"
    return {"value": round(n * cb / el, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n} steps x {cb} images ({'the full per-GPU batch' if cb == batch else 'a bounded sample of the per-GPU batch'}) "
                      f"at {size}, {what}; {el:.1f}s"}


def vgg19_features_():
    from dgan.zoo import vgg19_features
    return vgg19_features(1)


if __name__ == "__main__":
    main()
