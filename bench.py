"""Benchmark: train rays/s of the ScratchNerf mip-NeRF step on MI355X (BASELINE.json `metric`).

One step = both levels forward (stratified + hierarchical sampling, fused frustum/IPE/8x256 MLP,
integrator) + fused loss gradient + both levels backward (integrator adjoint, MLP dX chain,
weight-gradient GEMMs) + (N>1) RCCL all-reduce of the flat gradient arena + fused Adam.
Workload at N=1 = BASELINE.json configs[1]: Lego-shaped synthetic 800x800 batches of 1024 rays,
128 + 128 samples, 8x256 MLP, fp32.  At N>1 the default is configs[3]: a 65536-ray global batch
sharded over the N GPUs (strong scaling; each shard micro-batched in 8192-ray calls accumulated
into one gradient), with the N=1 line also carrying the same 65536-ray batch on one GPU
(`config4_1gpu`), the denominator of SURVEY §8(e)'s scaling ratio.  Inputs are pre-staged in HBM
before the timed region.

    python bench.py [--gpus N --steps K --warmup W]                      (N = 1)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
    python bench.py --gpus N --single-process                            (one process, N devices)

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
PRECISIONS = {"f32": 0, "split": 1, "f16x2": 2, "f16split": 3, "f16": 4}  # NOF_PRECISION_*
# f16split: the f16x2 pieces in every contraction (weight gradients too) — 3 fp16 MFMAs per product
# f16: one fp16 MFMA per product (plain mixed precision): the dense fp16 peak
PEAKS = {"f32": PEAK_F32_TFLOPS, "split": PEAK_SPLIT_TFLOPS, "f16x2": PEAK_F16X2_TFLOPS, "f16split": PEAK_F16X2_TFLOPS,
         "f16": PEAK_BF16_TFLOPS}
DTYPES = {"f32": "f32", "split": "f32 (bf16x3 split MFMA)", "f16x2": "f16x2 (fp16 hi+lo, 3 MFMAs; perf mode, 2e-3)",
          "f16split": "f32 via fp16 hi+lo in every contraction (3 MFMAs per product; 1e-5 parity, fp16 range)",
          "f16": "f16 (fp16 operands, fp32 accumulation, 1 MFMA per product; perf mode: outputs 2e-3, gradients "
                 "per tensor vs fp64 2e-3, W0/b0 6e-3 (measured 4.9e-3), tests/conftest.py f16_grad_tol)"}
PEAK_HBM_GBS = 8000.0
# weight-gradient operands per sample per level, each needed once per launch (fp16 in the f16x2 mode):
# activations IPE 96 + view PE 27 + h0..h7 8x256 + h9 128 = 2299, deltas 8x256 + d9 128 + the heads'
# dz_sigma 1 and dz_rgb 3 = 2180 (the stored blocks add 33 zero rows: not counted)
WGRAD_VALUES = 2299 + 2180
WGRAD_BYTES_PER_VALUE = {"f32": 4, "split": 4, "f16x2": 2, "f16split": 4, "f16": 2}
# algorithmic HBM bytes per sample per level of the F16 MLP kernels (mlp_f16.hip, fp16 blocks):
#   forward writes act_in 128 x 2 + h0..h7 8 x 256 x 2 + h9 128 x 2 + ReLU masks 9 x 32 + zhead 16 + sigma,
#   rgb 16 = 4928; backward writes delta 8 x 256 x 2 + delta9x 132 x 2 = 4360 and reads the masks 288,
#   zhead 16, dsigma / drgb 16 = 4680; weight gradients read every stored operand once (WGRAD_VALUES x 2)
KERNEL_BYTES_PER_SAMPLE = {"f16": {"mlp_fwd": 4928, "mlp_bwd": 4680, "wgrad": WGRAD_VALUES * 2}}
# BASELINE configs[0]'s network (4x128, one 128-wide view layer, PE 16 / 4): the any-shape fp32 path
CONFIG0_NET = dict(net_depth=4, net_width=128, net_depth_condition=1, net_width_condition=128, skip_layer=4,
                   min_deg_point=0, max_deg_point=16, deg_view=4)


def net_macs(net):
    """(forward, dX, dW) MACs per sample of a network (the layer list of accelerated.cpp / MLPcpp:131-154):
    forward and dW = every weight; dX = every weight row block that multiplies a hidden activation."""
    D, W, Dc, Wc = net["net_depth"], net["net_width"], net["net_depth_condition"], net["net_width_condition"]
    pos, dirs, skip = 6 * (net["max_deg_point"] - net["min_deg_point"]), 3 * (2 * net["deg_view"] + 1), net["skip_layer"]
    w = pos * W + sum(W * (W + (pos if l % skip == 0 else 0)) for l in range(1, D)) + W + Wc * (W + dirs) \
        + (Dc - 1) * Wc * Wc + 3 * Wc
    dx = (D - 1) * W * W + W + Wc * W + (Dc - 1) * Wc * Wc + 3 * Wc
    return w, dx, w
INTEGRATOR_FWD_B = lambda S: S * (12 + 4 + 4) + (S + 1) * 4 + 12 + 12  # rgb, sigma, w | t | d | C  (3100 @128)
INTEGRATOR_BWD_B = lambda S: 12 + S * (12 + 4) + (S + 1) * 4 + 12 + S * (12 + 4)  # 4636 @128


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--global-batch", type=int, default=None,
                   help="rays per step over all GPUs (default: 1024 at N=1 = configs[1]; 65536 at N>1 = configs[3], "
                        "strong scaling; LLFF: 512 per GPU = configs[4]'s per-GPU shape)")
    p.add_argument("--rays", type=int, default=None, help="rays per GPU per step (weak scaling: global = N x rays)")
    p.add_argument("--micro-batch", type=int, default=8192,
                   help="rays per get_gradient call; a larger shard is micro-batched and accumulated")
    p.add_argument("--single-process", action="store_true",
                   help="one process drives --gpus devices (nof_dp_init_all, grouped all-reduce) instead of one "
                        "process per GPU")
    p.add_argument("--no-config4", action="store_true", help="skip the N=1 configs[3] (65536-ray) measurement")
    p.add_argument("--no-config5", action="store_true",
                   help="skip the configs[4] leg (4096 LLFF rays x 256+256, f16x2, at every N)")
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
    p.add_argument("--cpu-seconds", type=float, default=20.0, help="target CPU-baseline work (both legs)")
    a = p.parse_args()
    if a.rays is not None:
        if a.global_batch is not None:
            p.error("--rays and --global-batch are exclusive")
        a.global_batch = a.rays * a.gpus
    a.global_batch_fixed = a.rays is None  # strong scaling unless the per-GPU size was given
    return a


def host_cpus():
    """(nproc, affinity, cgroup CPU quota or None, CPU model) of this host."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(math.ceil(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return os.cpu_count() or 1, aff, quota, model


def cpu_baseline(samples, target_s, net=None):
    """Oracle = faithful scalar C++ restatement of MipNerfModel.GetGradient (MNcs:99-200) + the Adam
    step (TrainState.cs:25-37 / AF:403-416), float, on a bounded sample of the same workload (BASELINE.md
    §2): once single-threaded (the C# path is single-threaded) and once OpenMP over rays on every host
    CPU this process may use (affinity, capped by a cgroup CPU quota when one is set)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from nof import synth

    nproc, aff, quota, model = host_cpus()
    spec = O.Spec() if net is None else O.Spec(D=net["net_depth"], W=net["net_width"], Dc=net["net_depth_condition"],
                                               Wc=net["net_width_condition"], skip=net["skip_layer"],
                                               min_deg=net["min_deg_point"], max_deg=net["max_deg_point"],
                                               deg_view=net["deg_view"])
    P0 = O.glorot_init(spec, 0x5EED0002)

    def timed(n, threads, seed):
        r = synth.blender_rays(n, seed=seed)
        P = P0.copy()
        m = np.zeros_like(P)
        v = np.zeros_like(P)
        t0 = time.perf_counter()
        out = O.step(spec, P, r, samples=tuple(samples), seed=seed, nthreads=threads, dtype=np.float32,
                     want=("grads",))
        O.adam_step(P, out["grads"], m, v, 5e-4, 1)
        return time.perf_counter() - t0

    def leg(threads, budget):
        probe = max(1, threads // 2)
        dt = timed(probe, threads, 99)
        n = max(threads, int(probe * budget / max(dt, 1e-3)) // threads * threads)
        dt = timed(n, threads, 100)
        return n, dt

    threads = min(aff, quota) if quota else aff
    n1, dt1 = leg(1, target_s * 0.4)
    nN, dtN = leg(threads, target_s * 0.6)
    step = f"one full step (both levels fwd + loss + bwd + Adam), {samples[0]}+{samples[1]} samples, float"
    return {"value": round(nN / dtN, 2), "unit": "rays/s", "cores": threads, "kind": "port",
            "sample": f"{nN} rays, {step}, OpenMP over rays on {threads} threads: {dtN:.1f} s",
            "single_thread": {"value": round(n1 / dt1, 3), "unit": "rays/s", "cores": 1,
                              "sample": f"{n1} rays, {step}: {dt1:.1f} s"},
            "host": {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota, "cpu_model": model}}


def profile_table(name):
    """profiles/<name> written by tools/pmc_summary.py from the committed rocprofv3 passes ({} if absent)."""
    f = os.path.join(ROOT, "profiles", name)
    try:
        return json.load(open(f)) if os.path.exists(f) else {}
    except (OSError, ValueError):
        return {}


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
    # HBM bytes per fwd + bwd pair from the committed PMC passes (tools/profile_r02.sh integrator leg)
    pmc = profile_table("pmc_traffic.json")
    tf, tb = pmc.get("render_fwd_integrator"), pmc.get("render_bwd_integrator")
    traffic = tf + tb if (tf is not None and tb is not None and S == 128 and n == 1 << 20) else None
    for name, v in (("render_fwd", tf), ("render_bwd", tb)):
        out[name]["traffic"] = v if traffic is not None else None
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4), "traffic": traffic, "algorithmic_bytes": tot_b,
            "workload": f"{n} rays x {S} samples, render fwd+bwd", "kernels": out}


def api_path(torch, nof, synth, dev, n, samples, prec, steps=20, warmup=3):
    """The reference's own boundary, host buffers in (PCIe-inclusive): MipNerfModel hands host arrays
    to AcceleratedMipNeRF::GetGradient (MNcpp:52-84 copies them to the device) and its output-gradient
    callback uploads the host pixels through AcceleratedGradientCalculator (AGC:19-33), then Adam.
    Same workload as the headline; the arrays are fresh host (pageable) numpy buffers each step, as
    a C# caller's managed arrays would be.  Reported beside `value`, never as it."""
    seed = 0x5EED0002
    m = nof.AcceleratedMipNeRF(device=dev.index, max_rays=n, num_samples=samples, seed=seed,
                               stream=torch.cuda.current_stream(dev).cuda_stream, precision=PRECISIONS[prec])
    opt = nof.AcceleratedAdamOptimizer(m.GetLayerSizes(), m.config)
    calc = nof.AcceleratedGradientCalculator(n, m.config)
    batches = [synth.blender_rays(n, seed=7000 + i) for i in range(2)]

    def step(k):
        r = batches[k % 2]
        m.set_rng(seed, k, 0)
        cb = lambda comp, level, msum, lm: calc.get_output_gradient(comp, r["pix"], lm, msum, level)
        grads = m.GetGradient(r["o"], r["d"], r["radius"], r["near"], r["far"], r["lossmult"], cb)
        opt.step(m.mlp.allParams, grads, nof.learning_rate_decay(k + 1))

    for k in range(warmup):
        step(k)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(warmup, warmup + steps):
        step(k)
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    calc.close()
    opt.close()
    m.close()
    h2d = n * (3 + 3 + 1 + 1 + 1 + 1) * 4 + len(samples) * n * 3 * 4
    return {"value": round(n * steps / dt, 1), "unit": "rays/s", "ms_per_step": round(dt * 1e3 / steps, 4),
            "steps": steps, "h2d_bytes_per_step": h2d,
            "path": "GetGradient(host arrays) + output-gradient callback (host pixels) + Adam, precision " + prec}


def render_throughput(torch, nof, synth, dev, prec, n=8192, samples=(128, 128), reps=10):
    """Evaluation path (MipNerfModel.Call, MNcs:36-97): the deterministic two-level
    render — forward-only MLP kernels, integrator with distance / accumulation, resampling — of
    device-resident rays, rays/s."""
    m = nof.AcceleratedMipNeRF(device=dev.index, max_rays=n, num_samples=samples, seed=0x5EED0002,
                               stream=torch.cuda.current_stream(dev).cuda_stream, precision=PRECISIONS[prec])
    r = synth.blender_rays(n, seed=77)
    t = {k: torch.from_numpy(r[k]).to(dev) for k in ("o", "d", "radius", "near", "far")}
    go = lambda: m.render_device(n, t["o"], t["d"], t["radius"], t["near"], t["far"], False)
    go()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        go()
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    m.close()
    return {"workload": f"deterministic two-level render of {n} Lego-shaped rays x {'+'.join(map(str, samples))} "
                        f"samples (forward only), precision {prec}", "value": round(n * reps / dt, 1),
            "unit": "rays/s", "ms_per_call": round(dt * 1e3 / reps, 4)}


def psnr_vs_ref(torch, nof, synth, dev, prec, n=64, steps=40, samples=(128, 128), n_eval=256):
    """Part of the cpu_baseline leg.  The metric's "PSNR vs ref": the HIP path and the oracle's float restatement of the reference
    (MipNerfModel.GetGradient MNcs:99-200 + the Adam step AF:403-416, the reference's CPU path in
    float) train from the same Glorot init on the same batches and Philox samples for `steps` steps;
    then both render a held-out batch deterministically (MipNerfModel.Call, MNcs:36-97) and the fine
    level's PSNR (MseToPsnr, MipHelpers.cs:672) of each is reported.  LR: LearningRateDecay without
    the 2500-step warm-up delay, so that a short run moves the weights."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    seed = 0x5EED0003
    spec = O.Spec()
    _, aff, quota, _ = host_cpus()
    threads = min(aff, quota) if quota else aff
    m = nof.AcceleratedMipNeRF(device=dev.index, max_rays=max(n, n_eval), num_samples=samples, seed=seed,
                               stream=torch.cuda.current_stream(dev).cuda_stream, precision=PRECISIONS[prec])
    opt = nof.AcceleratedAdamOptimizer(m.GetLayerSizes(), m.config)
    P = O.glorot_init(spec, seed)
    mo, vo = np.zeros_like(P), np.zeros_like(P)
    lr = lambda k: nof.learning_rate_decay(k, lr_delay_steps=0)
    t_ref = 0.0
    for k in range(steps):
        r = synth.blender_rays(n, seed=600 + k)
        d = {kk: torch.from_numpy(v).to(dev) for kk, v in r.items()}
        m.set_rng(seed, k, 0)
        g = m.get_gradient_device(n, d["o"], d["d"], d["radius"], d["near"], d["far"], d["lossmult"], d["pix"],
                                  float(np.sum(r["lossmult"], dtype=np.float32)))
        opt.step(m.mlp.allParams, g, lr(k + 1))
        t0 = time.perf_counter()
        out = O.step(spec, P, r, samples=tuple(samples), seed=seed, step_idx=k, ray_base=0, nthreads=threads,
                     dtype=np.float32, want=("grads",))
        O.adam_step(P, out["grads"], mo, vo, lr(k + 1), k + 1)
        t_ref += time.perf_counter() - t0
    torch.cuda.synchronize(dev)
    held = synth.blender_rays(n_eval, seed=999)
    c_gpu = m.render_rays(held, randomized=False)[-1]["comp_rgb"]
    ref = O.step(spec, P, held, samples=tuple(samples), seed=seed, randomized=False, nthreads=threads,
                 dtype=np.float32, want=("C",))
    pptr, cnt = m.mlp.flat_params()
    p_gpu = nof.to_numpy(pptr, (cnt,))
    psnr = lambda c: float(-10.0 * np.log10(np.mean((np.asarray(c, np.float64) - held["pix"]) ** 2)))
    res = {"psnr_hip": round(psnr(c_gpu), 4), "psnr_ref": round(psnr(ref["C"][-1]), 4),
           "params_rel_l2": float(np.linalg.norm(p_gpu - P) / np.linalg.norm(P)),
           "ref": "oracle float restatement of MipNerfModel.GetGradient + Adam (the reference's CPU path)",
           "training": f"{steps} steps x {n} rays x {'+'.join(map(str, samples))} samples, precision {prec}",
           "eval": f"{n_eval} held-out rays, deterministic render, fine level", "ref_cpu_s": round(t_ref, 1)}
    res["delta_db"] = round(res["psnr_hip"] - res["psnr_ref"], 4)
    opt.close()
    m.close()
    return res


def workload_name(a, B):
    if a.scene == "llff":
        return "BASELINE configs[4] per-GPU shape" if (B // a.gpus, a.samples) == (512, [256, 256]) else "LLFF-shaped"
    if a.samples == [128, 128] and B == 65536:
        return "BASELINE configs[3]"
    if a.samples == [128, 128] and B == 1024 * a.gpus:
        return "BASELINE configs[1]"
    return "BASELINE configs[2]" if a.samples == [64, 128] else "Lego-shaped"


def chunks(n, m):
    """[lo, hi) micro-batches of at most m rays covering n."""
    return [(lo, min(n, lo + m)) for lo in range(0, n, m)]


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    import nof
    from nof import synth
    from nof.dp import BucketedAllReduce, NativeDP, params_checksum

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    single = a.single_process
    if single and world != 1:
        raise SystemExit("--single-process drives every GPU from one process: do not launch it with torch.distributed")
    if not single and world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 via torch.distributed.run "
                         "(or --single-process)")
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

    G = a.gpus  # data-parallel width (ranks, or devices of the single process)
    B = a.global_batch or (512 * G if a.scene == "llff" else 1024 if G == 1 else 65536)
    if B % G:
        raise SystemExit(f"--global-batch {B} does not split over {G} GPUs")
    shard = B // G
    micro = min(a.micro_batch, shard)
    samples = a.samples
    seed = 0x5EED0002
    msum_global = float(B)  # lossmult = 1 everywhere: sum over all shards (D14, DP-global)
    devs = list(range(G)) if single else [dev_idx]
    ranks = list(range(G)) if single else [rank]

    # pre-staged synthetic batches per device (views of a 100-pose Lego-shaped scene), global ray ids
    def stage(r, d, n=shard, scene=None):
        out = []
        for i in range(2):
            h = (synth.llff_rays if (scene or a.scene) == "llff" else synth.blender_rays)(n, seed=1000 * r + i)
            out.append({k: torch.from_numpy(v).to(torch.device("cuda", d)) for k, v in h.items()})
        return out

    pools = [stage(r, d) for r, d in zip(ranks, devs)]

    native = None
    if single and G > 1:
        native = NativeDP.init_all(devs)
    elif world > 1 and a.dp == "native":  # C-ABI RCCL communicator; the id travels over torch.distributed
        obj = [NativeDP.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        native = [NativeDP.init_rank(obj[0], world, rank, dev_idx)]

    def measure(prec, B_run=None, steps=None, warmup=None, timers_on=True, scene=None, smp=None, net=None):
        """W untimed + K timed training steps of one precision mode over the global batch (each
        rank's shard in micro-batches accumulated into one gradient, one all-reduce), then a short
        untimed pass with every kernel class event-timed (the per-kernel breakdown); returns
        (s, timing, psnr, in_sync).  Inside the timed region only the MLP kernel classes (mlp_fwd,
        mlp_bwd, wgrad: the roofline kernel is among them) are bracketed by hipEvents: each event
        pair costs the dependent launch sequence a few us (measured 1.5 % of the f32 step and 4 % of
        the f16x2 step with every kernel class timed)."""
        B_run = B_run or B
        smp = list(smp or samples)
        sh = B_run // G
        mb = min(a.micro_batch, sh)
        steps = steps or a.steps
        warmup = a.warmup if warmup is None else warmup
        pl = pools if (sh == shard and scene in (None, a.scene)) else \
            [stage(r, d, sh, scene) for r, d in zip(ranks, devs)]
        models, opts, bucketed = [], [], []
        for r, d in zip(ranks, devs):
            st = torch.cuda.current_stream(torch.device("cuda", d)).cuda_stream
            m = nof.AcceleratedMipNeRF(device=d, max_rays=mb, num_samples=smp, seed=seed, stream=st,
                                       precision=PRECISIONS[prec], **(net or {}))
            models.append(m)
            opts.append(nof.AcceleratedAdamOptimizer(m.GetLayerSizes(), m.config))
        if world > 1 and native is None:  # torch.distributed: bucketed, overlapped with the backward
            bucketed = [BucketedAllReduce(models[0], dev, allreduce=allreduce)]
        if native is not None and not single:
            native[0].attach(models[0])  # RCCL buckets on the library's internal comm stream
        cs = chunks(sh, mb)
        try:  # the communicator is detached and the models closed whatever happens

            def step(k):
                for i, (r, m) in enumerate(zip(ranks, models)):
                    b = pl[i][k % 2]
                    for j, (lo, hi) in enumerate(cs):
                        m.set_rng(seed, k, r * sh + lo)  # global ray ids: sharding never changes a sample
                        m.get_gradient_device(hi - lo, b["o"][lo:hi], b["d"][lo:hi], b["radius"][lo:hi],
                                              b["near"][lo:hi], b["far"][lo:hi], b["lossmult"][lo:hi], b["pix"][lo:hi],
                                              msum_global, accumulate=j > 0, publish=j == len(cs) - 1)
                if single and G > 1:
                    NativeDP.allreduce_grads_all(native, models)
                for m, o in zip(models, opts):
                    o.step(m.mlp.allParams, m.mlp.allGradients, nof.learning_rate_decay(k + 1))
                if native is not None:
                    for nd in native:  # failure detection, one step behind (the host queues the next step
                        nd.step_end()  # meanwhile): an RCCL error or a stall raises instead of hanging

            def sync_all():
                if native is not None:
                    for nd in native:
                        nd.wait()  # the last step's all-reduces (bounded)
                for d in devs:
                    torch.cuda.synchronize(d)

            for k in range(warmup):
                step(k)
            sync_all()
            if world > 1:
                dist.barrier()
            # the three MLP kernel classes are event-timed live (the roofline kernel is the one that takes
            # the most time per step, which depends on the mode): 6 event pairs per step
            timers = os.environ.get("NOF_BENCH_TIMERS", "mlp_fwd,mlp_bwd,wgrad")
            models[0].enable_timing(timers_on, timers=timers.split(",") if timers != "all" else None)
            sync_all()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            for k in range(warmup, warmup + steps):
                step(k)
            sync_all()
            if world > 1:
                dist.barrier()
            dt = time.perf_counter() - t0
            live = models[0].read_timing()
            timing = {}
            kb = min(5, steps) if timers_on else 0
            if kb:  # per-kernel breakdown: a few more steps with every kernel class timed (outside the clock)
                # one untimed step first: read_timing synchronised, and the first timed class (pack) would
                # otherwise measure the idle GPU waiting for the host's first launch
                step(warmup + steps)
                models[0].enable_timing(True)
                for k in range(warmup + steps + 1, warmup + steps + 1 + kb):
                    step(k)
                timing = {name: (ms * steps / kb, cnt * steps // kb) for name, (ms, cnt) in models[0].read_timing().items()}
                for name, v in live.items():  # the live (timed-region) figures where they were taken
                    if v[1]:
                        timing[name] = v
                models[0].enable_timing(False)
            in_sync = None
            if world > 1 or (single and G > 1):
                sync_all()
                # DP invariant: identical all-reduced gradients + identical Adam -> every
                # rank holds bitwise-identical parameters; compare a checksum's max and min over ranks
                sums = []
                for m, d in zip(models, devs):
                    pptr, P = m.mlp.flat_params()
                    sums.append(params_checksum(nof.device_tensor(pptr, (P,), device=torch.device("cuda", d))).to(dev))
                cs_ = torch.cat(sums)
                hi, lo = cs_.max().reshape(1), (-cs_.min()).reshape(1)
                if world > 1:
                    t = torch.tensor([dt], device=dev, dtype=torch.float64)
                    allreduce(t, op=dist.ReduceOp.MAX)
                    dt = float(t.item())
                    allreduce(hi, op=dist.ReduceOp.MAX)
                    allreduce(lo, op=dist.ReduceOp.MAX)
                in_sync = bool(hi.item() == -lo.item())
            # fine-level PSNR of the last micro-batch (MseToPsnr, MipHelpers.cs:672)
            last = pl[0][(warmup + steps + kb - (0 if kb else 1)) % 2]
            lo_, hi_ = cs[-1]
            comp = models[0].level_numpy(len(smp) - 1)["comp_rgb"]
            mse = float(np.mean((comp - last["pix"][lo_:hi_].cpu().numpy()) ** 2))
            psnr = -10.0 * math.log10(max(mse, 1e-12))
        finally:
            for bk in bucketed:
                bk.close()
            if native is not None and not single:
                native[0].attach(None)
            for o, m in zip(opts, models):
                o.close()
                m.close()
        return dt, timing, psnr, in_sync

    def summarize(prec, dt, timing, sh=shard, smp=None, steps=None):
        steps = steps or a.steps
        ms_step = dt * 1e3 / steps
        M = [sh * s for s in (smp or samples)]
        flop = {"mlp_fwd": 2 * MACS_FWD * sum(M), "mlp_bwd": 2 * MACS_DX * sum(M), "wgrad": 2 * MACS_DW * sum(M)}
        kernels = {}
        for name, (ms, cnt) in timing.items():
            if cnt:
                kernels[name] = {"ms_per_step": round(ms / steps, 4), "launches_per_step": cnt // steps,
                                 "avg_launch_ms": round(ms / cnt, 4)}
        # algorithmic HBM bytes of the MLP kernels where they are an HBM stream as much as an MFMA
        # workload (the F16 mode): achieved GB/s beside the MFMA fraction of each
        for k, bps in KERNEL_BYTES_PER_SAMPLE.get(prec, {}).items():
            if k in kernels:
                b_launch = bps * sum(M) / kernels[k]["launches_per_step"]
                gbs = b_launch / (kernels[k]["avg_launch_ms"] * 1e-3) / 1e9
                kernels[k].update({"bytes_per_launch": b_launch, "achieved_gbs": round(gbs, 1),
                                   "hbm_frac": round(gbs / PEAK_HBM_GBS, 4)})
        dom = max((k for k in flop if k in kernels), key=lambda k: kernels[k]["ms_per_step"])
        fl_launch = flop[dom] / kernels[dom]["launches_per_step"]
        achieved = fl_launch / (kernels[dom]["avg_launch_ms"] * 1e-3) / 1e12
        mlp_ms = sum(kernels[k]["ms_per_step"] for k in flop if k in kernels)
        mlp_tf = sum(flop.values()) / (mlp_ms * 1e-3) / 1e12
        peak = PEAKS[prec]
        # committed rocprofv3 evidence (profiles/, tools/profile_r02.sh + tools/pmc_summary.py): HBM bytes
        # and MFMA-busy fraction per launch of the same kernels in the same configuration
        key = lambda k: k + ("" if prec == "f32" else "_" + prec)
        traffic = profile_table("pmc_traffic.json").get(key(dom))
        busy = profile_table("pmc_mfma.json")
        for k in kernels:
            if busy.get(key(k)) is not None:
                kernels[k]["mfma_busy"] = busy[key(k)]
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 2), "peak": peak,
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": traffic,
                "flop_per_launch": fl_launch, "mfma_busy": busy.get(key(dom))}
        if dom == "wgrad":
            # the weight-gradient launch streams every stored activation and delta once: in the f16
            # modes that stream, not the MFMAs, binds it — report the roofline that binds
            b_launch = WGRAD_VALUES * WGRAD_BYTES_PER_VALUE[prec] * sum(M) / kernels[dom]["launches_per_step"]
            gbs = b_launch / (kernels[dom]["avg_launch_ms"] * 1e-3) / 1e9
            hbm = {"bound": "hbm", "kernel": dom, "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                   "frac": round(gbs / PEAK_HBM_GBS, 4), "traffic": traffic, "bytes_per_launch": b_launch,
                   "mfma": {k: roof[k] for k in ("achieved", "peak", "unit", "frac", "mfma_busy")}}
            if hbm["frac"] > roof["frac"]:
                roof = hbm
        return ms_step, kernels, {
            "roofline": roof,
            "mlp_all_kernels": {"achieved": round(mlp_tf, 2), "unit": "TFLOP/s", "frac": round(mlp_tf / peak, 4)},
        }

    dt, timing, psnr, in_sync = measure(a.precision)
    rays_per_s = B * a.steps / dt
    alts = []
    lead = rank == 0
    if world == 1 and G == 1 and not a.no_alt:
        alts = [(p,) + measure(p) for p in PRECISIONS if p != a.precision]
    cfg4 = None
    llff = None
    if lead and world == 1 and G == 1 and a.scene == "blender" and not a.no_alt:
        # north_star's "rays/sec on synthetic LLFF-shape batches": the same step on forward-facing NDC
        # rays (the MLP work per sample does not depend on the ray distribution)
        l_dt, _, l_psnr, _ = measure(a.precision, steps=20, warmup=3, timers_on=False, scene="llff")
        llff = {"workload": f"LLFF-shaped (forward-facing, NDC) {B}-ray batches x {'+'.join(map(str, samples))} "
                            "samples", "value": round(B * 20 / l_dt, 1), "unit": "rays/s",
                "ms_per_step": round(l_dt * 1e3 / 20, 4), "steps": 20, "precision": a.precision}
    if lead and world == 1 and G == 1 and not a.no_config4 and B != 65536 and a.scene == "blender" \
            and samples == [128, 128]:
        # SURVEY §8(e)'s scaling denominator: config 4's 65536-ray global batch on this one GPU,
        # micro-batched into 8192-ray calls accumulated into one gradient, one Adam step per batch
        # 10 timed steps of ~0.4 s: a sustained stretch of full-GPU work (also what the driver's
        # utilisation sampler can see)
        c_steps = 10
        c_dt, _, _, _ = measure(a.precision, B_run=65536, steps=c_steps, warmup=1, timers_on=False)
        cfg4 = {"workload": "BASELINE configs[3] on 1 GPU: 65536-ray global batch x 128+128 samples, 8 micro-batches "
                            "of 8192 rays accumulated, one Adam step", "value": round(65536 * c_steps / c_dt, 1),
                "unit": "rays/s", "ms_per_step": round(c_dt * 1e3 / c_steps, 3), "steps": c_steps, "warmup": 1}

    cfg3 = None
    if lead and world == 1 and G == 1 and a.scene == "blender" and samples == [128, 128] and not a.no_alt:
        # BASELINE configs[2]: mip-NeRF coarse + fine with 64 + 128 hierarchical samples (the coarse level
        # stratified, the fine level resampled from it), same batch, same mode, its own live roofline
        c3_smp = [64, 128]
        c3_dt, c3_timing, c3_psnr, _ = measure(a.precision, smp=c3_smp)
        c3_ms, c3_kernels, c3_roof = summarize(a.precision, c3_dt, c3_timing, smp=c3_smp)
        c3_tf = 2 * (MACS_FWD + MACS_DX + MACS_DW) * shard * sum(c3_smp) / (c3_ms * 1e-3) / 1e12
        cfg3 = {"workload": f"BASELINE configs[2]: {B}-ray batches x 64+128 hierarchical samples (mip-NeRF "
                            f"coarse + fine), 8x256 MLP fwd/bwd + Adam", "value": round(B * a.steps / c3_dt, 1),
                "unit": "rays/s", "ms_per_step": round(c3_ms, 4), "steps": a.steps, "warmup": a.warmup,
                "precision": a.precision, "dtype": DTYPES[a.precision], **c3_roof,
                "roofline_step": {"bound": "mfma", "achieved": round(c3_tf, 2), "peak": PEAKS[a.precision],
                                  "unit": "TFLOP/s", "frac": round(c3_tf / PEAKS[a.precision], 4)},
                "kernels": c3_kernels, "psnr_fine": round(c3_psnr, 3)}

    cfg0 = None
    if lead and world == 1 and G == 1 and a.scene == "blender" and not a.no_alt:
        # BASELINE configs[0] (the reference's CPU-only plumbing case: 4096 rays x 64 samples, 4x128 MLP) on
        # the HIP path: the any-shape fp32 network path (generic.hip), coarse 64 + fine 64 samples
        z_B, z_smp = 4096, (64, 64)
        z_dt, _, z_psnr, _ = measure("f32", B_run=z_B, steps=20, warmup=3, timers_on=False, smp=z_smp, net=CONFIG0_NET)
        z_tf = 2 * sum(net_macs(CONFIG0_NET)) * z_B * sum(z_smp) / (z_dt / 20) / 1e12
        cfg0 = {"workload": f"BASELINE configs[0] on the GPU: {z_B}-ray batches x 64+64 samples, 4x128 MLP "
                            "(any-shape fp32 path: one MFMA GEMM launch per layer) fwd/bwd + Adam",
                "value": round(z_B * 20 / z_dt, 1), "unit": "rays/s", "ms_per_step": round(z_dt * 1e3 / 20, 4),
                "steps": 20, "warmup": 3, "dtype": "f32",
                "roofline_step": {"bound": "mfma", "achieved": round(z_tf, 2), "peak": PEAK_F32_TFLOPS,
                                  "unit": "TFLOP/s", "frac": round(z_tf / PEAK_F32_TFLOPS, 4),
                                  "macs_per_sample": net_macs(CONFIG0_NET)},
                "psnr_fine": round(z_psnr, 3)}

    cfg5 = None
    if a.scene == "blender" and not a.no_config5:
        # BASELINE configs[4] (north_star's "rays/sec on synthetic LLFF-shape batches at 1, 2, 4 and 8
        # GPUs"): 4096 forward-facing NDC rays x 256 + 256 samples per step over all N GPUs (512 per
        # GPU at N = 8), fp16 pieces on MFMA (the f16x2 perf mode), one all-reduce per step — at every N
        c_B = 4096
        if c_B % G == 0:
            c_dt, _, _, c_sync = measure("f16x2", B_run=c_B, steps=20, warmup=3, timers_on=False, scene="llff",
                                         smp=(256, 256))
            # the whole step's algorithmic MLP work per GPU against the f16x2 3-MFMA ceiling
            step_tf = 2 * (MACS_FWD + MACS_DX + MACS_DW) * (c_B // G) * 512 / (c_dt / 20) / 1e12
            cfg5 = {"workload": f"BASELINE configs[4]: LLFF-shaped (forward-facing, NDC) {c_B}-ray global batch x "
                                f"256+256 samples, {c_B // G} rays per GPU, f16x2 perf mode (fp16 pieces on MFMA)",
                    "value": round(c_B * 20 / c_dt, 1), "unit": "rays/s", "n_gpus": G,
                    "ms_per_step": round(c_dt * 1e3 / 20, 4), "steps": 20, "warmup": 3, "scaling": "strong",
                    "dtype": DTYPES["f16x2"],
                    "roofline_step": {"bound": "mfma", "achieved": round(step_tf, 2), "peak": PEAK_F16X2_TFLOPS,
                                      "unit": "TFLOP/s per GPU", "frac": round(step_tf / PEAK_F16X2_TFLOPS, 4),
                                      "note": "whole step (sampling, integrator, all-reduce and Adam included) "
                                              "over the MLP's algorithmic FLOP"}}
            if c_sync is not None:
                cfg5["params_in_sync"] = c_sync
            # the same batch in the plain fp16 mode (one fp16 MFMA per product: configs[4]'s "fp16
            # activations on MFMA" taken literally), against the dense fp16 peak
            if not a.no_alt:
                f_dt, _, _, f_sync = measure("f16", B_run=c_B, steps=20, warmup=3, timers_on=False, scene="llff",
                                             smp=(256, 256))
                f_tf = 2 * (MACS_FWD + MACS_DX + MACS_DW) * (c_B // G) * 512 / (f_dt / 20) / 1e12
                cfg5["f16"] = {"value": round(c_B * 20 / f_dt, 1), "unit": "rays/s", "ms_per_step": round(f_dt * 1e3 / 20, 4),
                               "dtype": DTYPES["f16"],
                               "roofline_step": {"bound": "mfma", "achieved": round(f_tf, 2), "peak": PEAKS["f16"],
                                                 "unit": "TFLOP/s per GPU", "frac": round(f_tf / PEAKS["f16"], 4)}}
                if f_sync is not None:
                    cfg5["f16"]["params_in_sync"] = f_sync

    result = None
    if lead:
        ms_step, kernels, roof = summarize(a.precision, dt, timing)
        strong = G > 1 and a.global_batch_fixed and a.scene == "blender"
        result = {
            "metric": METRIC, "value": round(rays_per_s, 1), "unit": "rays/s", "n_gpus": G, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None, "dtype": DTYPES[a.precision],
            "data": "synthetic (Lego-shaped 800x800, 100 poses)" if a.scene == "blender"
                    else "synthetic (forward-facing LLFF-shaped 800x800, NDC)",
            "config": {"workload": f"{workload_name(a, B)}: {B}-ray global batch x {'+'.join(map(str, samples))} "
                                   f"samples, 8x256 MLP fwd/bwd + Adam",
                       "global_batch": B, "rays_per_gpu": shard, "micro_batch": micro,
                       "micro_batches_per_step": len(chunks(shard, micro)), "samples": samples,
                       "parallelism": f"dp{G}", "precision": a.precision,
                       "allreduce": (("native (single process, grouped)" if single else
                                      "native (bucketed, overlapped)" if a.dp == "native" else
                                      "torch.distributed (bucketed, overlapped)") if G > 1 else None)},
            **roof,
            # the whole step per GPU (sampling, integrator, all-reduce, Adam included) over the MLP's
            # algorithmic FLOP: the scaling runs' roofline figure
            "roofline_step": {"bound": "mfma",
                              "achieved": round(2 * (MACS_FWD + MACS_DX + MACS_DW) * shard * sum(samples)
                                                / (ms_step * 1e-3) / 1e12, 2),
                              "peak": PEAKS[a.precision], "unit": "TFLOP/s per GPU"},
            "kernels": kernels,
            "psnr_fine": round(psnr, 3),
        }
        rs_ = result["roofline_step"]
        rs_["frac"] = round(rs_["achieved"] / rs_["peak"], 4)
        if G > 1:
            result["params_in_sync"] = in_sync
            if world > 1 and backend != "nccl":
                result["rehearsal"] = f"{backend}: {world} ranks on {torch.cuda.device_count()} GPU(s), not a scaling run"
        if llff:
            result["llff_1gpu"] = llff
        if cfg0:
            result["config0"] = cfg0
        if cfg3:
            result["config3"] = cfg3
        if cfg4:
            result["config4_1gpu"] = cfg4
        if cfg5:
            result["config5"] = cfg5
        if alts:  # the other precision modes, same workload (split: same 1e-5 parity; f16x2: 2e-3)
            result["alt_precision"] = []
            for aprec, adt, atiming, apsnr, _ in alts:
                ams, akernels, aroof = summarize(aprec, adt, atiming)
                entry = {"precision": aprec, "dtype": DTYPES[aprec], "value": round(B * a.steps / adt, 1),
                         "unit": "rays/s", "ms_per_step": round(ams, 4), **aroof,
                         "kernels": {k: v["avg_launch_ms"] for k, v in akernels.items()}, "psnr_fine": round(apsnr, 3)}
                if aprec in KERNEL_BYTES_PER_SAMPLE:  # each MLP kernel: MFMA fraction and achieved GB/s
                    fl = {"mlp_fwd": MACS_FWD, "mlp_bwd": MACS_DX, "wgrad": MACS_DW}
                    entry["kernel_rooflines"] = {
                        k: {"avg_launch_ms": v["avg_launch_ms"],
                            "mfma_frac": round(2 * fl[k] * B * sum(samples) / v["launches_per_step"]
                                               / (v["avg_launch_ms"] * 1e-3) / 1e12 / PEAKS[aprec], 4),
                            "achieved_gbs": v["achieved_gbs"], "hbm_frac": v["hbm_frac"],
                            "bytes_per_launch": v["bytes_per_launch"]}
                        for k, v in akernels.items() if "achieved_gbs" in v}
                result["alt_precision"].append(entry)
        if world == 1 and G == 1 and a.scene == "blender" and B <= 8192:
            result["api_path_pcie"] = api_path(torch, nof, synth, dev, B, samples, a.precision)
            result["render_1gpu"] = render_throughput(torch, nof, synth, dev, a.precision, samples=tuple(samples))
        if not a.no_integrator and world == 1 and G == 1:
            result["roofline_integrator"] = integrator_roofline(torch, nof, dev)
        if not a.no_cpu_baseline and world == 1 and G == 1:
            result["cpu_baseline"] = cpu_baseline(samples, a.cpu_seconds)
            if cfg0:  # configs[0]'s own case: the CPU restatement of the reference path on its 4x128 net
                cfg0["cpu_baseline"] = cpu_baseline((64, 64), a.cpu_seconds * 0.25, net=CONFIG0_NET)
            # same leg (the oracle runs only here): the reference's float CPU path trained beside the
            # HIP path on identical batches -> the metric's "PSNR vs ref"
            result["psnr_vs_ref"] = psnr_vs_ref(torch, nof, synth, dev, a.precision, samples=samples)
        print(json.dumps(result), flush=True)
    if native is not None:
        for nd in native:
            nd.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
