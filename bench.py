"""Benchmark: train rays/s of the ScratchNerf mip-NeRF step on MI355X (BASELINE.json `metric`).

One step = both levels forward (stratified + hierarchical sampling, fused frustum/IPE/8x256 MLP,
integrator) + fused loss gradient + both levels backward (integrator adjoint, MLP dX chain,
weight-gradient GEMMs) + (N>1) RCCL all-reduce of the flat gradient arena + fused Adam.
Workload = BASELINE.json configs[1]: Lego-shaped synthetic 800x800 batches, 1024 rays per GPU,
128 + 128 samples, 8x256 MLP, fp32.  Inputs are pre-staged in HBM before the timed region.

    python bench.py [--gpus N --steps K --warmup W]                      (N = 1)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line.  `roofline` covers the dominant kernel, timed live with hipEvents
on the library's stream inside the timed region; `cpu_baseline` times the oracle's faithful
C++ restatement of MipNerfModel.GetGradient on the host (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nerf-or-nothing_amd"))

METRIC = "train rays/sec (128 samples/ray, 8×256 MLP) at 1/2/4/8 MI355X; PSNR vs ref"
# algorithmic work per sample per level (SURVEY.md §8d / BASELINE.md §3)
MACS_FWD = 544768
MACS_DX = 492160
MACS_DW = 544768
PEAK_F32_TFLOPS = 157.3   # MI355X fp32 MFMA dense (= packed-fp32 VALU), MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 2516.6  # MI355X bf16 dense MFMA (no sparsity)
# split mode issues 6 bf16 MFMAs per fp32 product (mlp_common.h), so its fp32-equivalent ceiling is 1/6;
# the f16x2 perf mode issues 3 fp16 MFMAs (same dense rate as bf16) per product
PEAK_SPLIT_TFLOPS = round(PEAK_BF16_TFLOPS / 6, 1)
PEAK_F16X2_TFLOPS = round(PEAK_BF16_TFLOPS / 3, 1)
PRECISIONS = {"f32": 0, "split": 1, "f16x2": 2}  # NOF_PRECISION_*
PEAKS = {"f32": PEAK_F32_TFLOPS, "split": PEAK_SPLIT_TFLOPS, "f16x2": PEAK_F16X2_TFLOPS}
DTYPES = {"f32": "f32", "split": "f32 (bf16x3 split MFMA)", "f16x2": "f16x2 (fp16 hi+lo, 3 MFMAs; perf mode, 2e-3)"}
PEAK_HBM_GBS = 8000.0
INTEGRATOR_FWD_B = lambda S: S * (12 + 4 + 4) + (S + 1) * 4 + 12 + 12  # rgb, sigma, w | t | d | C  (3100 @128)
INTEGRATOR_BWD_B = lambda S: 12 + S * (12 + 4) + (S + 1) * 4 + 12 + S * (12 + 4)  # 4636 @128


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--rays", type=int, default=1024, help="rays per GPU per step")
    p.add_argument("--samples", type=int, nargs="+", default=[128, 128])
    p.add_argument("--scene", choices=["blender", "llff"], default="blender",
                   help="synthetic ray distribution: Lego-shaped 800x800 views (configs 2-4) or forward-facing "
                        "LLFF NDC rays (config 5: --scene llff --rays 512 --samples 256 256 --precision f16x2)")
    p.add_argument("--precision", choices=list(PRECISIONS), default="f32",
                   help="MLP contraction arithmetic: fp32 MFMA, fp32 operands as bf16x3 split MFMAs (same 1e-5 "
                        "parity), or the f16x2 perf mode (fp16 hi+lo, parity 2e-3)")
    p.add_argument("--no-alt", action="store_true", help="skip the other precision modes' secondary measurements")
    p.add_argument("--dp", choices=["torch", "native"], default="torch",
                   help="N>1 gradient all-reduce: torch.distributed (RCCL) or the C ABI's nof_dp_* (RCCL)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-integrator", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline work")
    return p.parse_args()


def cpu_baseline(samples, target_s):
    """Oracle = faithful scalar C++ restatement of MipNerfModel.GetGradient (MNcs:99-200), float,
    OpenMP over rays on this host; bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from nof import synth

    cores = min(16, os.cpu_count() or 1)
    spec = O.Spec()
    P = O.glorot_init(spec, 0x5EED0002)
    probe_n = cores
    r = synth.blender_rays(probe_n, seed=99)
    t0 = time.perf_counter()
    O.step(spec, P, r, samples=tuple(samples), seed=1, nthreads=cores, dtype=np.float32, want=("grads",))
    dt = time.perf_counter() - t0
    n = max(cores, int(probe_n * max(1.0, (target_s - dt) / max(dt, 1e-3))) // cores * cores)
    r = synth.blender_rays(n, seed=100)
    t0 = time.perf_counter()
    O.step(spec, P, r, samples=tuple(samples), seed=2, nthreads=cores, dtype=np.float32, want=("grads",))
    dt = time.perf_counter() - t0
    import platform
    model = platform.processor()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": n / dt, "unit": "rays/s", "cores": cores, "kind": "port",
            "sample": f"{n} rays x ({samples[0]}+{samples[1]}) samples, one full step (fwd+loss+bwd), float, "
                      f"OpenMP over rays, {dt:.1f} s on {model}"}


def integrator_roofline(torch, nof, dev, n=1 << 20, S=128, reps=5):
    """HBM roofline of the integrator fwd/bwd on an integrator-only 2^20 x 128 batch."""
    g = torch.Generator(device=dev).manual_seed(3)
    sigma = torch.rand((n, S), device=dev, generator=g) * 5
    rgb = torch.rand((n, S, 3), device=dev, generator=g)
    t = torch.sort(torch.rand((n, S + 1), device=dev, generator=g) * 4 + 2, dim=1).values
    d = torch.randn((n, 3), device=dev, generator=g)
    C = torch.empty((n, 3), device=dev)
    w = torch.empty((n, S), device=dev)
    gr = torch.randn((n, 3), device=dev, generator=g)
    ds = torch.empty((n, S), device=dev)
    dc = torch.empty((n, S, 3), device=dev)
    call = nof._lib.call
    fwd = lambda: call("nof_kernel_render", n, S, sigma.data_ptr(), rgb.data_ptr(), t.data_ptr(), d.data_ptr(), 1,
                       C.data_ptr(), w.data_ptr(), None)
    bwd = lambda: call("nof_kernel_render_grad", n, S, sigma.data_ptr(), rgb.data_ptr(), t.data_ptr(), d.data_ptr(),
                       1, C.data_ptr(), gr.data_ptr(), None, None, 0.0, 1.0, ds.data_ptr(), dc.data_ptr(), None)
    out = {}
    for name, fn, b in (("render_fwd", fwd, INTEGRATOR_FWD_B(S)), ("render_bwd", bwd, INTEGRATOR_BWD_B(S))):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gbs = b * n / (ms * 1e-3) / 1e9
        out[name] = {"ms": ms, "bytes_per_ray": b, "achieved": gbs, "frac": gbs / PEAK_HBM_GBS}
    tot_b = (INTEGRATOR_FWD_B(S) + INTEGRATOR_BWD_B(S)) * n
    tot_ms = out["render_fwd"]["ms"] + out["render_bwd"]["ms"]
    ach = tot_b / (tot_ms * 1e-3) / 1e9
    del sigma, rgb, t, d, C, w, gr, ds, dc
    torch.cuda.empty_cache()
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": None,
            "workload": f"{n} rays x {S} samples, render fwd+bwd", "kernels": out}


def workload_name(a):
    if a.scene == "llff":
        return "BASELINE configs[4] per-GPU shape" if (a.rays, a.samples) == (512, [256, 256]) else "LLFF-shaped"
    if (a.rays, a.samples) == (1024, [128, 128]):
        return "BASELINE configs[1]"
    return "BASELINE configs[2]" if a.samples == [64, 128] else "Lego-shaped"


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import nof
    from nof import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 via torch.distributed.run")
    # NOF_BENCH_DIST_BACKEND=gloo rehearses the N > 1 launch path (sharding, global sum of loss
    # multipliers, barriers, max-over-ranks timing) with several ranks on one GPU: the all-reduces go
    # through host memory, so its timings are not a scaling measurement.  Default: nccl (= RCCL).
    backend = os.environ.get("NOF_BENCH_DIST_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        raise SystemExit(f"NOF_BENCH_DIST_BACKEND={backend}: nccl or gloo")
    dev_idx = local if backend == "nccl" else local % torch.cuda.device_count()
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    def allreduce(t, op=dist.ReduceOp.SUM):
        if backend == "nccl":
            dist.all_reduce(t, op=op)
        else:  # rehearsal: through host memory
            h = t.cpu()
            dist.all_reduce(h, op=op)
            t.copy_(h)

    n = a.rays
    samples = a.samples
    stream = torch.cuda.current_stream(dev).cuda_stream
    seed = 0x5EED0002
    # pre-staged synthetic batches (views of a 100-pose Lego-shaped scene; shard = disjoint views)
    pool = []
    for i in range(4):
        r = (synth.llff_rays if a.scene == "llff" else synth.blender_rays)(n, seed=1000 * rank + i)
        pool.append({k: torch.from_numpy(v).to(dev) for k, v in r.items()})
    msum_global = float(n * world)  # lossmult = 1 everywhere: sum over all shards (D14, DP-global)

    native = None
    if world > 1 and a.dp == "native":  # C-ABI RCCL communicator; the id travels over torch.distributed
        from nof.dp import NativeDP

        obj = [NativeDP.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        native = NativeDP.init_rank(obj[0], world, rank, dev_idx)

    def measure(prec):
        """W untimed + K timed training steps of one precision mode, then a short untimed pass with
        every kernel class event-timed (the per-kernel breakdown); returns (s, timing, psnr, in_sync).
        Inside the timed region only the dominant kernel (mlp_fwd, the roofline kernel) is bracketed
        by hipEvents: each event pair costs the dependent launch sequence a few us (measured 1.5 % of
        the f32 step and 4 % of the f16x2 step with every kernel timed)."""
        model = nof.AcceleratedMipNeRF(device=dev_idx, max_rays=n, num_samples=samples, seed=seed,
                                       stream=stream, precision=PRECISIONS[prec])
        model.set_rng(seed, 0, rank * n)  # global ray ids: sharding never changes a sample
        opt = nof.AcceleratedAdamOptimizer(model.GetLayerSizes(), model.config)
        params = model.mlp.allParams
        gptr, P = model.mlp.flat_grads()
        grad_view = nof.device_tensor(gptr, (P,), device=dev)

        def step(k):
            b = pool[k % len(pool)]
            grads = model.get_gradient_device(n, b["o"], b["d"], b["radius"], b["near"], b["far"],
                                              b["lossmult"], b["pix"], msum_global)
            if native is not None:
                native.allreduce_grads(model, stream)
            elif world > 1:
                allreduce(grad_view)  # sum of per-shard gradient sums (no averaging: L is a sum)
            opt.step(params, grads, nof.learning_rate_decay(k + 1))

        for k in range(a.warmup):
            step(k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        timers = os.environ.get("NOF_BENCH_TIMERS", "mlp_fwd")
        model.enable_timing(True, timers=timers.split(",") if timers != "all" else None)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for k in range(a.warmup, a.warmup + a.steps):
            step(k)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        live = model.read_timing()
        # per-kernel breakdown: a few more steps with every kernel class timed (outside the clock)
        kb = min(5, a.steps)
        model.enable_timing(True)
        for k in range(a.warmup + a.steps, a.warmup + a.steps + kb):
            step(k)
        timing = {name: (ms * a.steps / kb, cnt * a.steps // kb) for name, (ms, cnt) in model.read_timing().items()}
        for name, v in live.items():  # the live (timed-region) figures where they were taken
            if v[1]:
                timing[name] = v
        model.enable_timing(False)
        in_sync = None
        if world > 1:
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            allreduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
            # DP invariant: identical all-reduced gradients + identical Adam -> every
            # rank holds bitwise-identical parameters; compare a checksum's max and min over ranks
            pptr, P = model.mlp.flat_params()
            pv = nof.device_tensor(pptr, (P,), device=dev).view(torch.int32).to(torch.int64)
            cs = (pv * torch.arange(1, P + 1, device=dev, dtype=torch.int64)).sum().reshape(1)
            hi, lo = cs.clone(), -cs
            allreduce(hi, op=dist.ReduceOp.MAX)
            allreduce(lo, op=dist.ReduceOp.MAX)
            in_sync = bool(hi.item() == -lo.item())
        # fine-level PSNR of the last step's batch (MseToPsnr, MipHelpers.cs:672)
        last = pool[(a.warmup + a.steps + kb - 1) % len(pool)]
        comp = model.level_numpy(len(samples) - 1)["comp_rgb"]
        mse = float(np.mean((comp - last["pix"].cpu().numpy()) ** 2))
        psnr = -10.0 * math.log10(max(mse, 1e-12))
        opt.close()
        model.close()
        return dt, timing, psnr, in_sync

    def summarize(prec, dt, timing):
        ms_step = dt * 1e3 / a.steps
        M = [n * s for s in samples]
        flop = {"mlp_fwd": 2 * MACS_FWD * sum(M), "mlp_bwd": 2 * MACS_DX * sum(M), "wgrad": 2 * MACS_DW * sum(M)}
        kernels = {}
        for name, (ms, cnt) in timing.items():
            if cnt:
                kernels[name] = {"ms_per_step": round(ms / a.steps, 4), "launches_per_step": cnt // a.steps,
                                 "avg_launch_ms": round(ms / cnt, 4)}
        dom = max((k for k in flop if k in kernels), key=lambda k: kernels[k]["ms_per_step"])
        fl_launch = flop[dom] / kernels[dom]["launches_per_step"]
        achieved = fl_launch / (kernels[dom]["avg_launch_ms"] * 1e-3) / 1e12
        mlp_ms = sum(kernels[k]["ms_per_step"] for k in flop if k in kernels)
        mlp_tf = sum(flop.values()) / (mlp_ms * 1e-3) / 1e12
        peak = PEAKS[prec]
        traffic = None
        tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tfile):
            try:
                traffic = json.load(open(tfile)).get(dom + ("" if prec == "f32" else "_" + prec))
            except (OSError, ValueError):
                traffic = None
        return ms_step, kernels, {
            "roofline": {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                         "flop_per_launch": fl_launch},
            "mlp_all_kernels": {"achieved": round(mlp_tf, 2), "unit": "TFLOP/s", "frac": round(mlp_tf / peak, 4)},
        }

    dt, timing, psnr, in_sync = measure(a.precision)
    rays_per_s = n * world * a.steps / dt
    alts = []
    if world == 1 and not a.no_alt:
        alts = [(p,) + measure(p) for p in PRECISIONS if p != a.precision]

    result = None
    if rank == 0:
        ms_step, kernels, roof = summarize(a.precision, dt, timing)
        result = {
            "metric": METRIC, "value": round(rays_per_s, 1), "unit": "rays/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": DTYPES[a.precision],
            "data": "synthetic (Lego-shaped 800x800, 100 poses)" if a.scene == "blender"
                    else "synthetic (forward-facing LLFF-shaped 800x800, NDC)",
            "config": {"workload": f"{workload_name(a)}: {n}-ray batches x {'+'.join(map(str, samples))} samples, "
                                   "8x256 MLP fwd/bwd + Adam",
                       "rays_per_gpu": n, "global_batch": n * world, "samples": samples,
                       "parallelism": f"dp{world}", "precision": a.precision,
                       "allreduce": a.dp if world > 1 else None},
            **roof,
            "kernels": kernels,
            "psnr_fine": round(psnr, 3),
        }
        if world > 1:
            result["params_in_sync"] = in_sync
            if backend != "nccl":
                result["rehearsal"] = f"{backend}: {world} ranks on {torch.cuda.device_count()} GPU(s), not a scaling run"
        if alts:  # the other precision modes, same workload (split: same 1e-5 parity; f16x2: 2e-3)
            result["alt_precision"] = []
            for aprec, adt, atiming, apsnr, _ in alts:
                ams, akernels, aroof = summarize(aprec, adt, atiming)
                result["alt_precision"].append({
                    "precision": aprec, "dtype": DTYPES[aprec], "value": round(n * a.steps / adt, 1),
                    "unit": "rays/s", "ms_per_step": round(ams, 4), **aroof,
                    "kernels": {k: v["avg_launch_ms"] for k, v in akernels.items()}, "psnr_fine": round(apsnr, 3)})
        if not a.no_integrator and world == 1:
            result["roofline_integrator"] = integrator_roofline(torch, nof, dev)
        if not a.no_cpu_baseline and world == 1:
            result["cpu_baseline"] = cpu_baseline(samples, a.cpu_seconds)
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
