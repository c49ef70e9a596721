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
PEAK_FP32_TFLOPS = 157.3      # MI355X dense FP32 (vector = MFMA), MI355X_MICROARCH.md
SR = 48000


TRAFFIC_FILE = os.path.join(REPO, "profiles", "conv_traffic.json")


def traffic_per_op(config: str, B: int, T: int):
    """HBM bytes per conv op from the committed rocprofv3 PMC passes
    (tools/profile_round.sh -> tools/rocprof_summary.py), for this exact
    workload only; null otherwise."""
    try:
        with open(TRAFFIC_FILE) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None
    if t.get("workload") != [config, B, T]:
        return None
    return t.get("bytes_per_op")


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
    ap.add_argument("--precision", default="f32", choices=["f32", "split16", "auto"],
                    help="conv/unit GEMM arithmetic (include/rave_amd.h RAVE_PREC_*)")
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
    model = RAVE(cfg, params, spk, device=dev, precision=a.precision)
    B, T = a.batch, a.samples
    Fz = T // cfg.hop
    x = torch.from_numpy(synth_batch(B, T, 1000 * rank)).to(dev)
    from rave_amd.distributed import ShardedRunner
    runner = ShardedRunner(model)          # encode -> RCCL all-gather of latents -> decode

    def step():
        return runner.step(x)[1]

    pe = model._encode_plan(B, T)
    pd = model._decode_plan(B, Fz)
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
        conv_ms = conv_fl = 0.0
        rows = []
        from rave_amd import _native as N
        n_conv = 0
        for plan, tm in ((pe, te), (pd, td)):
            for sym, lab, fl, ms in zip(plan.sym, plan.labels, plan.flops, tm):
                rows.append((lab, fl, ms))
                if sym[0] == N.OP_CONV:
                    conv_ms += ms
                    conv_fl += fl
                    n_conv += 1
        achieved = conv_fl / (conv_ms * 1e-3) / 1e12
        roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                "traffic": traffic_per_op(cfg.name, B, T),
                "kernel": "conv1d_mfma_kernel (+ its split-K reduce): all %d conv ops of one step, "
                          "fp32 MFMA 32x32x2" % n_conv,
                "flop_per_launch_avg": conv_fl / max(n_conv, 1),
                "avg_launch_ms": conv_ms / max(n_conv, 1),
                "event_ms_per_step": round(float(te.sum() + td.sum()), 4),
                "timing": "HIP events inside the conv dispatches, K steps after the timed pass"}
        if rank == 0:
            log(f"{'op':58s} {'GFLOP':>8s} {'ms':>8s} {'TFLOP/s':>8s}")
            for lab, fl, ms in rows:
                log(f"{lab[-58:]:58s} {fl / 1e9:8.3f} {ms:8.4f} {fl / max(ms, 1e-9) / 1e9:8.2f}")

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        cpu = cpu_baseline(cfg, params, spk, a.cpu_seconds, threads)

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "samples/s", "n_gpus": world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
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
