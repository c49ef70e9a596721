#!/usr/bin/env python3
"""Benchmark of the RAVE encode->decode hot path on MI355X.

Metric (BASELINE.json): audio samples/sec (48 kHz v2 encode+decode) and the
x-real-time factor.  Workload = BASELINE config 2: v2 non-causal
encode+decode of 16 clips x 65536 samples per GPU (synthetic audio,
random-init weights of the v2 architecture).  One step = RAVE.encode(x) on the
rank's 16 clips -> RCCL all-gather of the latents over all ranks -> RAVE.decode
of the rank's own latent shard.  Per-GPU work is fixed
as N grows ("scaling": "weak").

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

Rank 0 prints ONE JSON line; diagnostics go to stderr.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

METRIC = "audio samples/sec/GPU (48 kHz v2 encode+decode); × real-time factor"
PEAK_HBM_GBS = 8000.0         # MI355X HBM3E spec peak, MI355X_MICROARCH.md
PEAK_FP32_TFLOPS = 157.3      # MI355X dense FP32 MFMA (= vector rate), MI355X_MICROARCH.md
PEAK_F16_TFLOPS = 2516.6      # MI355X dense F16 MFMA (256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz)
# split16 issues three f16 MFMAs (hi*hi, hi*lo, lo*hi) per fp32 multiply-accumulate,
# so its ceiling in fp32-op FLOP is a third of the f16 peak
PEAK_SPLIT16_TFLOPS = round(PEAK_F16_TFLOPS / 3, 1)
SR = 48000

# GEMM-shaped kernel families of a step: name -> (kernels, peak in fp32-op TFLOP/s).
# The names match tools/rocprof_summary.py's grouping of rocprofv3 kernel rows.
FAMILIES = {
    "conv_f32": ("conv1d_mfma_kernel + conv1d_splitk_reduce_kernel, fp32 MFMA 32x32x2",
                 PEAK_FP32_TFLOPS),
    "conv_split16": ("conv1d_split_kernel + split_reduce_kernel, split-f16 MFMA 32x32x16 (3 per fp32 MAC)",
                     PEAK_SPLIT16_TFLOPS),
    "unit_f32": ("residual_unit_kernel, fp32 MFMA 32x32x2", PEAK_FP32_TFLOPS),
    "unit_split16": ("unit_split_kernel, split-f16 MFMA 32x32x16 (3 per fp32 MAC)", PEAK_SPLIT16_TFLOPS),
    "stack_split16": ("stack_split_kernel (3 residual units per launch), split-f16 MFMA 32x32x16",
                      PEAK_SPLIT16_TFLOPS),
    "pqmf_analysis": ("pqmf_analysis_kernel, fp32 MFMA 16x16x4", PEAK_FP32_TFLOPS),
    "pqmf_synthesis": ("pqmf_synthesis_kernel, fp32 MFMA 16x16x4", PEAK_FP32_TFLOPS),
}


def op_family(kind: int, scalars: dict) -> str:
    from rave_amd import _native as N
    prec = "split16" if scalars.get("precision", 0) == N.PREC_SPLIT16 else "f32"
    if kind == N.OP_CONV:
        return "conv_" + prec
    if kind == N.OP_UNIT:
        return "unit_" + prec
    if kind == N.OP_STACK:
        return "stack_split16"
    if kind == N.OP_PQMF_ANALYSIS:
        return "pqmf_analysis"
    if kind == N.OP_PQMF_SYNTHESIS:
        return "pqmf_synthesis"
    return "other"


TRAFFIC_FILE = os.path.join(REPO, "profiles", "traffic.json")


def traffic_per_launch(config: str, B: int, T: int, precision: str):
    """HBM bytes per op launch, per kernel family, from the committed rocprofv3
    PMC passes (tools/profile_round.sh -> tools/rocprof_summary.py), for this
    exact workload and precision only; None otherwise."""
    try:
        with open(TRAFFIC_FILE) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None
    if t.get("workload") != [config, B, T] or t.get("precision") != precision:
        return None
    return {k: v["bytes_per_launch"] for k, v in t.get("families", {}).items()}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synth_batch(B, T, seed0):
    n = np.arange(T)
    xs = []
    for b in range(B):
        rng = np.random.Generator(np.random.PCG64(seed0 + b))
        xs.append(0.3 * np.sin(2 * np.pi * 440 * n / SR) + 0.1 * rng.standard_normal(T))
    return np.stack(xs)[:, None, :].astype(np.float32)


def cpu_baseline(cfg, params, spk, seconds: float, threads: int):
    """The oracle (numpy float64 restatement, oracle/rave_oracle.py) on a bounded
    sample of the same workload: whole 65536-sample clips, repeated for about
    ``seconds`` of wall time, BLAS limited to ``threads`` threads."""
    from oracle.rave_oracle import Oracle
    from threadpoolctl import threadpool_limits
    o = Oracle(cfg, params, spk)
    x = synth_batch(1, 65536, 0)
    with threadpool_limits(limits=threads):
        o.forward(x)   # warm-up
        n, t0 = 0, time.perf_counter()
        while True:
            o.forward(x)
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    return {"value": n * 65536 / el, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{n} x v2 forward of one 65536-sample clip (numpy float64 oracle, "
                      f"{el:.1f} s wall, BLAS threads={threads})"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="clips per GPU")
    ap.add_argument("--samples", type=int, default=65536, help="samples per clip")
    ap.add_argument("--config", default="v2")
    ap.add_argument("--precision", default="auto", choices=["f32", "split16", "auto"],
                    help="conv/unit GEMM arithmetic (include/rave_amd.h RAVE_PREC_*); auto = the "
                         "faster of the two per op, timed when the plans are built")
    ap.add_argument("--tuning-in", help="JSON of RAVE.tuning() to reuse (no timing runs at plan build)")
    ap.add_argument("--tuning-out", help="write RAVE.tuning() here after the plans are built")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    a = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")

    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.weights import init_params, init_speaker

    cfg = rcfg.get_config(a.config)
    params = init_params(cfg, seed=0)
    spk = init_speaker(cfg, seed=0)
    tuning = None
    if a.tuning_in:
        with open(a.tuning_in) as fh:
            tuning = json.load(fh)
    model = RAVE(cfg, params, spk, device=dev, precision=a.precision, tuning=tuning)
    B, T = a.batch, a.samples
    Fz = T // cfg.hop
    x = torch.from_numpy(synth_batch(B, T, 1000 * rank)).to(dev)
    from rave_amd.distributed import ShardedRunner
    runner = ShardedRunner(model)          # encode -> RCCL all-gather of latents -> decode

    def step():
        return runner.step(x)[1]

    pe = model._encode_plan(B, T)
    pd = model._decode_plan(B, Fz)
    if a.tuning_out and rank == 0:
        with open(a.tuning_out, "w") as fh:
            json.dump(model.tuning(), fh)
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    profile = not a.no_profile
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        y = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total = world * B * T * a.steps
    value = total / el
    ms_step = 1e3 * el / a.steps
    if not torch.isfinite(y).all():
        raise RuntimeError("non-finite output")

    # ---------------------------------------------------------- roofline (HIP events per op)
    roof = None
    if profile:
        # Per-op timing over a second pass of the same K steps: the events ride
        # inside the kernels' own dispatch packets (hipExtLaunchKernelGGL, no
        # marker packets, no host syncs).  Kept out of the timed pass above,
        # whose wall time the event bookkeeping would stretch (~15 %).
        pe.profile(a.steps)
        pd.profile(a.steps)
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        te, ne = pe.op_times()
        td, nd = pd.op_times()
        pe.profile(0)
        pd.profile(0)
        if ne != a.steps or nd != a.steps:
            raise RuntimeError(f"profiled {ne}/{nd} runs, expected {a.steps}")
        te /= a.steps
        td /= a.steps
        rows = []
        fams: dict = {}
        for plan, tm in ((pe, te), (pd, td)):
            for sym, lab, fl, nb, ms in zip(plan.sym, plan.labels, plan.flops, plan.nbytes, tm):
                fam = op_family(sym[0], sym[2])
                rows.append((lab, fam, fl, nb, ms))
                if fam in FAMILIES:
                    f = fams.setdefault(fam, [0, 0.0, 0.0, 0.0])
                    f[0] += 1
                    f[1] += fl
                    f[2] += nb
                    f[3] += float(ms)
        traffic = traffic_per_launch(cfg.name, B, T, a.precision)

        def floor_ms(k):
            """(MFMA-bound, HBM-bound) time of a family's ops at the peaks, ms."""
            _, fl, nb, _ = fams[k]
            return fl / (FAMILIES[k][1] * 1e12) * 1e3, nb / (PEAK_HBM_GBS * 1e9) * 1e3

        def fam_line(k):
            n, fl, nb, ms = fams[k]
            kern, peak = FAMILIES[k]
            t_mfma, t_hbm = floor_ms(k)
            if t_hbm > t_mfma:        # the roof that binds this family at its algorithmic counts
                bound, ach, pk, unit = "hbm", nb / (ms * 1e-3) / 1e9, PEAK_HBM_GBS, "GB/s"
            else:
                bound, ach, pk, unit = "mfma", fl / (ms * 1e-3) / 1e12, peak, "TFLOP/s"
            return {"kernel": kern, "launches": n, "bound": bound, "achieved": round(ach, 3), "peak": pk,
                    "unit": unit, "frac": round(ach / pk, 4),
                    "tflops": round(fl / (ms * 1e-3) / 1e12, 3), "mfma_peak": peak,
                    "flop_per_launch_avg": fl / n, "bytes_per_launch_avg": nb / n, "avg_launch_ms": ms / n,
                    "traffic": (traffic or {}).get(k)}

        per = {k: fam_line(k) for k in sorted(fams)}
        # the dominant GEMM kernel family (largest share of the step) is the roofline line;
        # every family and the all-GEMM aggregate ride along
        dom = max(fams, key=lambda k: fams[k][3])
        tot_ms = sum(f[3] for f in fams.values())
        ideal_ms = sum(max(floor_ms(k)) for k in fams)
        d = per[dom]
        roof = {"bound": d["bound"], "achieved": d["achieved"], "peak": d["peak"], "unit": d["unit"],
                "frac": d["frac"], "traffic": d["traffic"],
                "kernel": f"{dom}: {d['kernel']} ({d['launches']} launches per step)",
                "flop_per_launch_avg": d["flop_per_launch_avg"],
                "bytes_per_launch_avg": d["bytes_per_launch_avg"], "avg_launch_ms": d["avg_launch_ms"],
                "families": per,
                "all_gemm_ops": {"ms_per_step": round(tot_ms, 4), "floor_ms_per_step": round(ideal_ms, 4),
                                 "frac": round(ideal_ms / tot_ms, 4)},
                "event_ms_per_step": round(float(te.sum() + td.sum()), 4),
                "timing": "HIP events inside each op's dispatches, K steps after the timed pass; "
                          "FLOP = algorithmic 2*MACs of the fp32 op; bytes = algorithmic (every "
                          "tensor and weight read or written once)"}
        if rank == 0:
            log(f"{'op':58s} {'family':14s} {'GFLOP':>8s} {'MB':>7s} {'ms':>8s} {'TFLOP/s':>8s} {'GB/s':>7s}")
            for lab, fam, fl, nb, ms in rows:
                ms_ = max(ms, 1e-9)
                log(f"{lab[-58:]:58s} {fam:14s} {fl / 1e9:8.3f} {nb / 1e6:7.2f} {ms:8.4f} "
                    f"{fl / ms_ / 1e9:8.2f} {nb / ms_ / 1e6:7.0f}")

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(cfg, params, spk, a.cpu_seconds, threads)

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "precision": {"f32": "exact-fp32 MFMA", "split16": "split-f16 (hi/lo) MFMA, fp32 accumulate",
                          "auto": "per op the faster of exact-fp32 MFMA and split-f16 (hi/lo) MFMA with "
                                  "fp32 accumulate; both meet the 1e-4 parity bound"}[a.precision],
            "data": "synthetic (440 Hz sine + N(0,0.1) noise; seeded random-init v2 weights)",
            "config": {"workload": f"{cfg.name} non-causal encode+decode, {B} x {T} samples per GPU "
                                   "(BASELINE configs[1])",
                       "global_batch": world * B, "samples_per_clip": T,
                       "parallelism": f"dp{world} (batch shards, RCCL all-gather of latents)"},
            "x_realtime": round(value / SR, 1),
            "per_gpu_samples_per_s": round(value / world, 1),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
