"""Benchmark: Model-A-7M CIFAR-100 32x32 training throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step = one full training iteration on a synthetic batch already resident in HBM:
autocast(bf16) forward through the HIP OutGridBlock kernels, CE(label smoothing 0.1), backward,
clip_grad_norm(1.0), fused AdamW, WarmupCosine — bs=512 per GPU (weak scaling).  The step runs
as a replayed hipGraph (ogv.train.Trainer, graphs=True; --eager for plain launches); for N>1 the
gradients are averaged by ~8 MB bucketed RCCL all_reduces recorded INSIDE the step's one graph, each
launched as soon as backward has produced its bucket (overlapping the rest of the backward;
--dp-flat: one flat all_reduce between two graphs, --dp-capture: one flat all_reduce captured at
the end of the graph).
Prints ONE JSON line on rank 0 with `roofline` (dominant kernel: HIP events around every launch
of it in one step — in graph mode an eager step right after the timed replays, since ROCm graphs
cannot hold timing events) and `cpu_baseline`
(the CPU oracle's train step on the host cores, bounded sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
PKG = ROOT / "outlook-grid-vision-transformer_amd"
sys.path.insert(0, str(PKG))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense bf16 MFMA peak (no 2:1 sparsity)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=512, help="per-GPU batch")
    ap.add_argument("--model", default="model_a_7m")
    ap.add_argument("--probe", default=None,
                    choices=["gemm_panel", "gemm_tiled", "sgemm", "wgrad", "gemm_fwd", "outlook_fwd", "outlook_bwd", "grid_fwd"],
                    help="kernel family whose launches feed `roofline` (default: the largest-time family of "
                         "the model's replayed step, DOMINANT below)")
    ap.add_argument("--eager", action="store_true", help="launch kernels one by one instead of graph replay")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=24.0)
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="ogv_set_option tuning switch (repeatable; see include/ogv.h)")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="launcher / process-group rehearsal on the CPU (gloo): every rank builds the model, "
                         "the Trainer broadcasts it and each step runs only the gradient all-reduce; no HIP kernels")
    ap.add_argument("--force-dp", action="store_true",
                    help="take the data-parallel path (process group, broadcast, per-step gradient all_reduce) at "
                         "N=1 too: a world-size-1 RCCL ('nccl') group on one GPU")
    ap.add_argument("--dp-capture", action="store_true",
                    help="graph mode with DP: capture ONE flat RCCL all_reduce at the end of the step's graph")
    ap.add_argument("--dp-flat", action="store_true",
                    help="graph mode with DP: graph A -> one flat all_reduce -> graph B instead of the default "
                         "bucketed all_reduces captured on a side stream during backward")
    ap.add_argument("--step-roofline", type=int, default=1,
                    help="1: time every C-ABI op of one eager step (after the timed region) for roofline.step")
    return ap.parse_args()


def launch_ranks(argv, n, cpu=False):
    """`--gpus N` (N > 1) started without a torchrun environment: start the N ranks ourselves --
    torch.distributed.run as a CHILD process (one process per GPU, rendezvous on 127.0.0.1) with
    the same arguments -- and return its exit code.  Runs before anything in this process touches
    the GPU (only the device count is read), so no initialised HIP context is carried into a fork
    or exec."""
    import socket
    import subprocess
    if not cpu:
        have = torch.cuda.device_count()     # does not initialise the GPU on this image
        if have < n:
            raise SystemExit(f"bench.py: --gpus {n} but only {have} HIP devices are visible")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"), *argv]
    return subprocess.call(cmd, env=env)


METRIC = {  # BASELINE.json configs[1..4]
    "model_a_7m": "training imgs/s Model-A-7M CIFAR-100 32x32",
    "model_a_14m_tin64": "training imgs/s Model-A-14M TinyImageNet-200 64x64",
    "model_a_22m_224": "training imgs/s Model-A-22M synthetic-ImageNet 224x224",
    "model_b_cifar100": "training imgs/s Model-B (OutlookerFrontGridNet) CIFAR-100 32x32",
}

# the largest-time kernel family of each workload's replayed step (rocprofv3 step breakdowns under
# profiles/: r02_head_step_breakdown.txt, r02_head_14m_step_breakdown.txt, r02_head_22m_step_breakdown.txt)
DOMINANT = {"model_a_7m": "gemm_panel", "model_a_14m_tin64": "wgrad", "model_a_22m_224": "wgrad",
            "model_b_cifar100": "gemm_panel"}

PROBE_KERNEL = {  # probe name -> kernel symbol(s) it times (rocprofv3 names)
    "gemm_panel": "ogv::pgemm_bf16_kernel<*> (pipelined panel GEMM: the Linear / 1x1-conv forward and "
                  "data-gradient launches at M < 65536 -- stages 1-3 of 7M; the largest-time kernel family "
                  "of the step)",
    "gemm_tiled": "ogv::gemm_bf16_kernel<*> (LDS-tiled MFMA GEMM: Linear / 1x1-conv launches routed to "
                  "neither the streaming nor the panel kernel, and the implicit-GEMM convs)",
    "wgrad": "ogv::wgrad2_bf16_kernel<*> (pipelined split-M; also wgrad_bf16 / swgrad_bf16 where planned) + its slab "
             "reduction (Linear / 1x1-conv weight gradients)",
    "outlook_bwd": "ogv::outlook_bwd_tile_kernel<*> (LDS-tiled outlook backward: the col2im fold as a gather + dlogits)",
    "sgemm": "ogv::sgemm_bf16_kernel<*> (persistent streaming projection GEMM: the Linear / 1x1-conv fwd and dgrad "
             "launches routed to it)",
    "gemm_fwd": "ogv::gemm_bf16_kernel<{128|64},{128|64},*,false,0,false> (Linear / 1x1-conv forward launches)",
    "outlook_fwd": "ogv::outlook_fwd_kernel",
    "grid_fwd": "ogv::grid_fwd_kernel",
}


def fwd_parity(device):
    """max|logits - reference logits| on the golden Model-A-7M B=2 case (reference output
    recorded from pablo-reyes8/outlook-grid-vision-transformer), fp32 and bf16-autocast."""
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import numpy as np
    import gen_params as gp
    from ogv.train import MODEL_CONFIGS, build_model
    z = np.load(ROOT / "tests" / "golden" / "model_a_7m_eval_b2.npz", allow_pickle=False)
    meta = json.loads(bytes(z["meta"]).decode())
    m = build_model(dict(type="model_a", num_classes=100, stem_dim=64, dpr_max=meta["dpr_max"],
                         stages=meta["stages"]))
    gp.fill_module(m, meta["seed"])
    m = m.to(device).eval()
    x = torch.from_numpy(gp.input_from_spec(meta["x"])).to(device).contiguous(memory_format=torch.channels_last)
    ref = torch.from_numpy(z["logits"]).double()
    out = {}
    with torch.no_grad():
        out["fp32"] = (m(x).double().cpu() - ref).abs().max().item()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out["bf16"] = (m(x).double().cpu() - ref).abs().max().item()
    out["ref_abs_max"] = ref.abs().max().item()
    out["bf16_rel"] = out["bf16"] / out["ref_abs_max"]
    # the reference's own CPU bf16-autocast forward (src/training/autocast.py:71-78) on the same
    # weights and input, recorded by running the reference (make_golden.py r3): its max|d| from the
    # reference's fp32 logits
    za = np.load(ROOT / "tests" / "golden" / "model_a_7m_eval_b2_autocast.npz", allow_pickle=False)
    out["bf16_reference_cpu_autocast"] = float(np.abs(za["logits_cpu_bf16_autocast"].astype(np.float64)
                                                      - za["logits"].astype(np.float64)).max())
    return out


def _host_threads():
    """Threads for the CPU baseline: the CPUs this process may run on (the box's CPU share:
    sched_getaffinity), capped by OMP_NUM_THREADS when the launcher sets it."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(seconds):
    """The oracle's fwd+CE+bwd+clip+AdamW, fp32, NCHW on the host cores (bounded), at the two
    batch sizes SURVEY §8d times the reference at: bs=64 (the host's best throughput) as three
    timed samples whose MEDIAN is `value` (single samples swung 57-85 imgs/s box to box), and one
    bs=8 sample (config 1) for context."""
    import statistics
    sys.path.insert(0, str(ROOT / "oracle"))
    sys.path.insert(0, str(ROOT / "tests" / "golden"))
    import gen_params as gp
    import ogv_oracle as orc
    from ogv.train import MODEL_CONFIGS
    cfg = MODEL_CONFIGS["model_a_7m"]
    threads = _host_threads()
    torch.set_num_threads(threads)
    samples = []
    per = seconds / 4
    for bs, reps in ((8, 1), (64, 3)):
        p = orc.make_params(orc.model_a_shapes(cfg["stages"], cfg["num_classes"], 3, cfg["stem_dim"]),
                            lambda k, s: gp.param_value(k, s, 7))
        opt = orc.make_optimizer(p)
        g = torch.Generator().manual_seed(7)
        x = torch.randn(bs, 3, 32, 32, generator=g)
        y = torch.randint(0, 100, (bs,), generator=g)
        for _ in range(2):
            orc.train_step(x, y, p, cfg["stages"], opt)
        for _ in range(reps):
            n, t0 = 0, time.perf_counter()
            while True:
                orc.train_step(x, y, p, cfg["stages"], opt)
                n += 1
                if time.perf_counter() - t0 > per:
                    break
            dt = time.perf_counter() - t0
            samples.append({"bs": bs, "steps": n, "seconds": round(dt, 2), "imgs_per_s": round(n * bs / dt, 2)})
    med = statistics.median(s["imgs_per_s"] for s in samples if s["bs"] == 64)
    return {"value": round(med, 2), "unit": "imgs/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(),
            "sample": f"Model-A-7M 32x32 fp32 fwd+CE+bwd+clip+AdamW (oracle restatement of the reference), "
                      f"~{per:.0f}s per sample after 2 warmup steps: bs=64 x3 (value = their median) and bs=8 x1; "
                      f"{threads} threads (this process's CPU affinity / OMP_NUM_THREADS)",
            "samples": samples}


def dry_run(args):
    """CPU rehearsal of the N-rank path (gloo): the launcher, the process group, the Trainer's
    start-up broadcast and the per-step flat gradient all-reduce of the real model's size.  Prints
    one JSON line on rank 0 with the world size the process group reports; no HIP kernel runs and
    no throughput is claimed (`value` null)."""
    from ogv.train import MODEL_CONFIGS, Trainer, build_model, setup_distributed
    rank, world, _, _ = setup_distributed(cpu=True)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the process group has {world} ranks")
    cfg = MODEL_CONFIGS[args.model]
    torch.manual_seed(7 + rank)          # a different init per rank: the broadcast must equalise them
    model = build_model({k: v for k, v in cfg.items() if k != "img"})
    trainer = Trainer(model, graphs=False, bucket_mb=0)
    with torch.no_grad():
        ck = torch.stack([sum(p.double().sum() for p in model.parameters())] * 2)
    ck[1] = -ck[1]
    ranks = [rank]
    if world > 1:
        dist.all_reduce(ck, op=dist.ReduceOp.MAX)         # max and -min of the parameter checksum
        ranks = [None] * world
        dist.all_gather_object(ranks, rank)
    flat = trainer.flat if world > 1 else torch.zeros(sum(p.numel() for p in model.parameters()) + 1)
    for _ in range(args.warmup):
        flat.fill_(rank + 1.0)
        if world > 1:
            trainer._allreduce()
    dist.barrier() if world > 1 else None
    t0 = time.perf_counter()
    for _ in range(args.steps):
        flat.fill_(rank + 1.0)
        if world > 1:
            trainer._allreduce()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    expect = world * (world + 1) / 2
    ok = bool((flat == expect).all()) if world > 1 else True
    if rank == 0:
        print(json.dumps({
            "metric": METRIC.get(args.model, args.model) + " [CPU dry run: launcher + gradient all-reduce only]",
            "value": None, "unit": "imgs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * t.item() / max(1, args.steps), 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "none (dry run)", "dry_run": True,
            "config": {"workload": f"{args.model} flat gradient all-reduce (gloo)", "parallelism": f"dp{world}",
                       "backend": dist.get_backend() if world > 1 else None},
            "ranks_reported": sorted(ranks), "allreduce_elems": flat.numel(), "allreduce_ok": ok,
            "params_broadcast_ok": bool(ck[0].item() == -ck[1].item())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(sys.argv[1:], args.gpus, cpu=args.cpu_dry_run))
    if args.cpu_dry_run:
        return dry_run(args)
    if args.probe is None:
        args.probe = DOMINANT.get(args.model, "gemm_panel")
    from ogv import functional as OF
    from ogv.train import MODEL_CONFIGS, Trainer, build_model, setup_distributed
    import ogv

    if args.force_dp and "WORLD_SIZE" not in os.environ:
        # a world-1 process group (env rendezvous on 127.0.0.1), set up before anything touches the GPU
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]), WORLD_SIZE="1",
                              RANK="0", LOCAL_RANK="0")
    rank, world, local, device = setup_distributed(force_group=args.force_dp)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE is {world}")
    torch.backends.cudnn.benchmark = True   # as the reference (src/training/autocast.py:8-17)
    assert device.type == "cuda", "bench.py needs a HIP device"
    ogv.load()
    for o in args.opt:
        name, val = o.split("=")
        if ogv._lib.load().ogv_set_option(name.encode(), int(val)) != 0:
            raise SystemExit(f"bench.py: unknown option {name}")
    cfg = MODEL_CONFIGS[args.model]
    torch.manual_seed(7)
    model = build_model({k: v for k, v in cfg.items() if k != "img"})
    model = model.to(device).to(memory_format=torch.channels_last)
    trainer = Trainer(model, total_steps=max(100, args.steps + args.warmup + 1), graphs=not args.eager,
                      capture_warmup=max(0, args.warmup - 1), force_dp=args.force_dp,
                      dp_capture_collective=args.dp_capture, dp_overlap=not args.dp_flat)

    B, S = args.batch, cfg["img"]
    g = torch.Generator(device=device).manual_seed(7 + rank)
    x = torch.randn(B, 3, S, S, device=device, generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, cfg["num_classes"], (B,), device=device, generator=g)

    for _ in range(max(0, args.warmup - 1)):
        trainer.step(x, y)
    trainer.step(x, y)       # last warmup step (graph mode: eager step on a side stream + capture)
    OF.probe_reset()
    if trainer.dp:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if not trainer.graphs:
            OF.probe_arm(args.probe)
        loss = trainer.step(x, y)
    torch.cuda.synchronize()
    if trainer.dp:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    OF.probe_disarm()
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    whatif = any(o.split("=")[0] in ("skip", "pg_dbg", "vp_dbg") and o.split("=")[1] != "0" for o in args.opt)
    assert whatif or torch.isfinite(loss).item(), "non-finite loss"   # (what-if timing runs leave outputs unwritten)
    # device memory of the benchmarked run (the reference logs the same two peaks every epoch,
    # src/training/train_full_model.py:19-20,184-185): warm-up + capture + the timed steps
    gib = float(2 ** 30)
    free_b, total_b = torch.cuda.mem_get_info(device)
    memory = {"peak_alloc_gib": round(torch.cuda.max_memory_allocated(device) / gib, 3),
              "peak_reserved_gib": round(torch.cuda.max_memory_reserved(device) / gib, 3),
              "device_total_gib": round(total_b / gib, 3),
              "device_used_gib_after_timing": round((total_b - free_b) / gib, 3)}
    memory["headroom_frac"] = round(1.0 - memory["peak_reserved_gib"] / memory["device_total_gib"], 4)
    if trainer.graphs:
        # the diagnostics below run eager steps: drop the recorded graph and return its private pool first,
        # so they never allocate beside it (22M at 224^2 came within 1.1 GB of the device that way, round 5)
        trainer.release_graphs()
        torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(device)
    if trainer.graphs:
        # ROCm graphs cannot carry timing events (torch: "External events are disallowed in rocm"), so
        # the probed kernel's launches are timed with HIP events in one eager step right after the
        # timed replays: same kernels, shapes and stream.
        OF.probe_reset()
        OF.probe_arm(args.probe)
        trainer._eager(x, y)
        OF.probe_disarm()
    probe = OF.probe_results()
    census = None
    if args.step_roofline:
        # SURVEY §8d's step-level roofline: every C-ABI op of one more eager step timed with HIP events
        # (same spin / overhead treatment as the probe), each against its algorithmic bytes / flops
        OF.census_reset()
        OF.census_arm()
        trainer._eager(x, y)
        OF.census_disarm()
        census = OF.census_results(HBM_PEAK_GBS, MFMA_PEAK_TFLOPS)
    memory["diagnostic_eager_peak_alloc_gib"] = round(torch.cuda.max_memory_allocated(device) / gib, 3)

    if rank == 0:
        value = world * B * args.steps / elapsed
        roof = None
        if probe and probe["achieved_GBs"]:
            traffic = None
            tf = ROOT / "profiles" / "pmc_traffic.json"
            if tf.exists():   # PMC passes of this workload (tools/gpu_measure.sh): 7M bs=512 under the probe's
                # name, any other workload under '<model>/bs<B>:<probe>'
                key = args.probe if (args.model == "model_a_7m" and B == 512) else f"{args.model}/bs{B}:{args.probe}"
                traffic = json.loads(tf.read_text()).get(key, {}).get("hbm_bytes_per_launch")
            ach = probe["achieved_GBs"]
            roof = {"probe": args.probe, "kernel": PROBE_KERNEL[args.probe], "bound": "hbm", "achieved": round(ach, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "algorithmic_bytes_per_launch": int(probe["bytes_per_launch"]),
                    "avg_launch_ms": round(probe["avg_ms"], 5), "launches": probe["n"],
                    "event_overhead_ms": round(probe["event_overhead_ms"], 5),
                    # the same launches' algorithmic flops against the dense bf16 MFMA peak (all the
                    # probed kernels sit far below the ~310 flop/B ridge, so this is small by construction)
                    "compute": {"achieved": round(probe["achieved_TFLOPs"], 2), "peak": MFMA_PEAK_TFLOPS,
                             "unit": "TFLOP/s", "frac": round(probe["achieved_TFLOPs"] / MFMA_PEAK_TFLOPS, 4),
                             "algorithmic_flops_per_launch": int(probe["flops_per_launch"])},
                    "timing": ("HIP events around each launch (a 40 us device spin queued ahead of each, so no host "
                               "launch gap is timed; raw intervals, nothing subtracted: they equal rocprofv3's kernel "
                               "durations, profiles/r03_final_probe_vs_trace.txt), " + ("eager step after the timed graph replays"
                                                           if trainer.graphs else "all timed steps"))}
        if roof is not None and census is not None:
            # clip + AdamW (ogv_clip_adamw: the norm pass reads g; the update pass reads p, g, m, v and writes
            # them back, g clipped in place): 36 B per fp32 parameter, priced at 40 B (the torch path's bytes)
            n_par = sum(p.numel() for p in trainer.params)
            opt_ms = 40.0 * n_par / (HBM_PEAK_GBS * 1e9) * 1e3
            bound_ms = census["bound_ms"] + opt_ms
            step_ms = 1e3 * elapsed / args.steps
            roof["step"] = {
                "definition": "sum over every C-ABI op of one train step of max(algorithmic bytes / 8 TB/s, "
                              "flops / 2.5 PFLOP/s) (SURVEY §8d), + the optimizer's 40 B/param at 8 TB/s",
                "algorithmic_bytes": int(census["bytes"] + 40 * n_par), "algorithmic_flops": int(census["flops"]),
                "bound_ms": round(bound_ms, 4), "ops": census["ops"],
                "native_ops_bound_ms": census["bound_ms"], "native_ops_measured_ms": census["measured_ms"],
                "frac_native_ops": census["frac"],          # Σ roofline time / Σ measured time over the native ops
                "frac_wall": round(bound_ms / step_ms, 4),   # bound_ms / the timed ms_per_step
                "families": census["families"]}
        out = {
            "metric": METRIC.get(args.model, args.model) + f" (bf16, bs={B}/GPU)",
            "value": round(value, 1), "unit": "imgs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16", "data": "synthetic (randn images, randint labels; random init)",
            "config": {"workload": f"{args.model} train step: fwd+CE(ls=0.1)+bwd+clip(1.0)+AdamW", "img_size": S,
                       "per_gpu_batch": B, "global_batch": B * world, "parallelism": f"dp{world}",
                       "execution": "hipGraph replay" if trainer.graphs else "eager launches",
                       "backend": trainer.backend or "none (single process, no collective)",
                       "dp_collective": (None if not trainer.dp else
                                         f"{len(trainer._gbuckets)} bucketed all_reduces captured in the step graph (on "
                                         "RCCL's stream), each launched as backward completes its bucket"
                                         if getattr(trainer, "dp_overlap", False) and hasattr(trainer, "_gbuckets") else
                                         "all_reduce captured in the step graph"
                                         if trainer.dp_capture_collective else
                                         "one flat all_reduce between graph A and graph B" if trainer.graphs else
                                         "bucketed async all_reduce during backward")},
            "roofline": roof,
            "peak_alloc_gib": memory["peak_alloc_gib"], "peak_reserved_gib": memory["peak_reserved_gib"],
            "memory": memory,
        }
        if world == 1 and not args.no_parity:
            out["fwd_max_abs_diff"] = fwd_parity(device)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
            out["gpu_over_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)
    if trainer.dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
