#!/usr/bin/env python3
"""Benchmark of the RAVE encode->decode hot path on MI355X.

Metric (BASELINE.json): audio samples/sec (48 kHz v2 encode+decode) and the
x-real-time factor.  Workload = BASELINE config 2: v2 non-causal
encode+decode of 16 clips x 65536 samples per GPU (synthetic audio,
random-init weights of the v2 architecture).  One step = RAVE.encode(x) on the
rank's 16 clips -> RCCL all-gather of the latents over all ranks -> RAVE.decode
of the rank's own latent shard.  Per-GPU work is fixed
as N grows ("scaling": "weak").

The headline ``value`` runs ``--precision f32_bf3`` (since round 4, late): fp32
arithmetic on every conv / unit GEMM with the committed launch choices
(profiles/tuning/) -- per op the faster of exact fp32 MFMA
(v_mfma_f32_32x32x2_f32) and, for the fused residual units, fp32 on the bf16
matrix cores with every operand split exactly into three bf16 parts (24
significand bits, the fp32 exponent range) and six of the nine cross products
(the three dropped are each below 2^-25 of the product), fp32 accumulation.
Its error against a float64 reference is within 1.5x (+1e-7 of the output
scale) of the exact-fp32 MFMA kernels' on the same inputs, and the two differ by
<= 1e-6 of the output scale (tests/test_gpu_parity.py::
test_residual_unit_bf16x3_is_fp32_class, test_conv_bf16x3_is_fp32_class).  The
same invocation then times, on the same input, ``f32_exact`` (``--precision
f32_tuned``: exact fp32 MFMA on every op) and ``split16_auto`` (per op the
faster of exact fp32 and split-f16 GEMMs on ~22-bit f16 hi/lo operands), each
with the max-abs difference of its output from the headline's.
``--precision f32_tuned`` / ``auto`` give the earlier layouts.  ``cpu_baseline`` is the
reference's module graph on torch fp32 CPU (oracle/torch_cpu.py) over the same
step.

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
# bf16x3 issues six bf16 MFMAs per fp32 multiply-accumulate (bf16 peak = f16 peak)
PEAK_BF3_TFLOPS = round(PEAK_F16_TFLOPS / 6, 1)
# (the bf16x3 decoder tail, since round 6 bf16x3 in its conv AND its synthesis,
# has the bf16x3 roof; round 5's tail mixed in an exact-fp32 synthesis)
# the bf16x3 encoder head mixes two roofs: its analysis (6 bands x 513 taps = 3078 MACs
# per frame) at the bf16x3 peak, its conv (64 x 6 x 7 = 2688 MACs per frame) at the fp32
# peak; its ceiling is the FLOP-weighted harmonic mean of the two
PEAK_HEAD_BF3_TFLOPS = round((3078 + 2688) / (3078 / PEAK_BF3_TFLOPS + 2688 / PEAK_FP32_TFLOPS), 1)
SR = 48000

# GEMM-shaped kernel families of a step: name -> (kernels, peak in fp32-op TFLOP/s).
# The names match tools/rocprof_summary.py's grouping of rocprofv3 kernel rows.
FAMILIES = {
    "conv_f32": ("conv1d_mfma_kernel / conv1d_ring_f32_kernel (+ split-K reduce), exact fp32 MFMA 32x32x2",
                 PEAK_FP32_TFLOPS),
    "conv_split16": ("conv1d_split_kernel + split_reduce_kernel, split-f16 MFMA 32x32x16 (3 per fp32 MAC)",
                     PEAK_SPLIT16_TFLOPS),
    "unit_f32": ("unit_ring_f32_kernel / residual_unit_kernel, exact fp32 MFMA 32x32x2", PEAK_FP32_TFLOPS),
    "unit_split16": ("unit_split_kernel, split-f16 MFMA 32x32x16 (3 per fp32 MAC)", PEAK_SPLIT16_TFLOPS),
    "conv_bf16x3": ("conv1d_bf3_kernel (+ split-K reduce), fp32 as exact bf16x3 operands, bf16 MFMA 32x32x16 "
                    "(6 per fp32 MAC)", PEAK_BF3_TFLOPS),
    "unit_bf16x3": ("unit_bf3_kernel, fp32 as exact bf16x3 operands, bf16 MFMA 32x32x16 (6 per fp32 MAC)",
                    PEAK_BF3_TFLOPS),
    "stack_split16": ("stack_split_kernel (3 residual units per launch), split-f16 MFMA 32x32x16",
                      PEAK_SPLIT16_TFLOPS),
    "stack_bf16x3": ("stack_bf3_kernel (3 residual units per launch), fp32 as exact bf16x3 operands, bf16 MFMA "
                     "32x32x16 (6 per fp32 MAC)", PEAK_BF3_TFLOPS),
    "pqmf_analysis_f32": ("pqmf_analysis_kernel, fp32 MFMA 16x16x4", PEAK_FP32_TFLOPS),
    "pqmf_synthesis_f32": ("pqmf_synthesis_kernel, fp32 MFMA 16x16x4", PEAK_FP32_TFLOPS),
    "pqmf_analysis_split16": ("pqmf_analysis_split_kernel, split-f16 MFMA 16x16x32 (3 per fp32 MAC)",
                              PEAK_SPLIT16_TFLOPS),
    "pqmf_synthesis_split16": ("pqmf_synthesis_split_kernel, split-f16 MFMA 16x16x32 (3 per fp32 MAC)",
                               PEAK_SPLIT16_TFLOPS),
    "head_split16": ("encoder_head_kernel: PQMF analysis (phase-packed) + EncoderV2's first conv, split-f16 "
                     "MFMA 16x16x32 / 32x32x16", PEAK_SPLIT16_TFLOPS),
    "tail_split16": ("decoder_tail_kernel: GeneratorV2's last conv + epilogue + PQMF synthesis, split-f16 "
                     "MFMA 32x32x16 / 16x16x32", PEAK_SPLIT16_TFLOPS),
    "head_f32": ("encoder_head_kernel<F32>: PQMF analysis (phase-packed) + EncoderV2's first conv, exact fp32 "
                 "MFMA 16x16x4 / 32x32x2", PEAK_FP32_TFLOPS),
    "tail_f32": ("decoder_tail_kernel<F32>: GeneratorV2's last conv + epilogue + PQMF synthesis, exact fp32 "
                 "MFMA 32x32x2 / 16x16x4", PEAK_FP32_TFLOPS),
    "tail_bf16x3": ("decoder_tail_kernel<BF16X3>: GeneratorV2's last conv in bf16x3 (bf16 MFMA 32x32x16, 6 per fp32 "
                    "MAC) + epilogue + PQMF synthesis in bf16x3 (MFMA 16x16x32, 6 per fp32 MAC; round 6)",
                    PEAK_BF3_TFLOPS),
    "head_bf16x3": ("encoder_head_kernel<BF16X3>: PQMF analysis (phase-packed) in bf16x3 (bf16 MFMA 16x16x32, 6 per "
                    "fp32 MAC) + EncoderV2's first conv in exact fp32 (MFMA 32x32x2)", PEAK_HEAD_BF3_TFLOPS),
}


def op_family(kind: int, precision: int) -> str:
    from rave_amd import _native as N
    prec = "split16" if precision == N.PREC_SPLIT16 else "f32"
    if kind in (N.OP_UNIT, N.OP_CONV, N.OP_STACK) and precision == N.PREC_BF16X3:
        return {N.OP_UNIT: "unit_", N.OP_CONV: "conv_", N.OP_STACK: "stack_"}[kind] + "bf16x3"
    if kind == N.OP_CONV:
        return "conv_" + prec
    if kind == N.OP_UNIT:
        return "unit_" + prec
    if kind == N.OP_STACK:
        return "stack_split16"
    if kind == N.OP_PQMF_ANALYSIS:
        return "pqmf_analysis_" + prec
    if kind == N.OP_PQMF_SYNTHESIS:
        return "pqmf_synthesis_" + prec
    if kind == N.OP_HEAD:
        return "head_bf16x3" if precision == N.PREC_BF16X3 else "head_" + prec
    if kind == N.OP_TAIL:
        return "tail_bf16x3" if precision == N.PREC_BF16X3 else "tail_" + prec
    return "other"


# committed PMC traffic per arithmetic mode (tools/profile_round.sh -> tools/rocprof_summary.py)
TRAFFIC_FILES = {"auto": os.path.join(REPO, "profiles", "traffic.json"),
                 "f32_tuned": os.path.join(REPO, "profiles", "traffic_f32_tuned.json"),
                 "f32_bf3": os.path.join(REPO, "profiles", "traffic_f32_bf3.json")}


def traffic_per_launch(config: str, B: int, T: int, precision: str):
    """HBM bytes per op launch, per kernel family, from the committed rocprofv3
    PMC passes (tools/profile_round.sh -> tools/rocprof_summary.py), for this
    exact workload and precision only; None otherwise."""
    if precision not in TRAFFIC_FILES:
        return None
    try:
        with open(TRAFFIC_FILES[precision]) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None
    if t.get("workload") != [config, B, T] or t.get("precision") != precision:
        return None
    return {k: v["bytes_per_launch"] for k, v in t.get("families", {}).items()}


def tuning_path(config: str, B: int, T: int, precision: str) -> str:
    """The committed launch-choice file of one workload and arithmetic mode."""
    return os.path.join(REPO, "profiles", "tuning", f"{config}_{B}x{T}_{precision}.json")


def tuning_hash(tuning) -> str:
    """sha256 (16 hex) of a RAVE.tuning() list, order-independent."""
    import hashlib
    rows = sorted(f"{k} {int(c)}" for k, c, _ in tuning)
    return hashlib.sha256("\n".join(rows).encode()).hexdigest()[:16]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synth_batch(B, T, seed0):
    n = np.arange(T)
    xs = []
    for b in range(B):
        rng = np.random.Generator(np.random.PCG64(seed0 + b))
        xs.append(0.3 * np.sin(2 * np.pi * 440 * n / SR) + 0.1 * rng.standard_normal(T))
    return np.stack(xs)[:, None, :].astype(np.float32)


def host_info() -> dict:
    """The host the CPU baseline ran on: CPU model, logical CPUs, 1-minute load."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        load = round(os.getloadavg()[0], 2)
    except OSError:
        load = None
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "loadavg_1min": load}


def usable_cpus() -> dict:
    """The CPUs this process may actually use: the affinity mask and the cgroup
    CPU quota (cgroup v2 cpu.max, or v1 cfs quota / period), beside the host's
    logical CPU count.  On the shared GPU hosts the quota (16 CPUs of a 256-CPU
    host) is what "all host cores" can mean for one process: 256 threads under
    a 16-CPU quota measured 51 s per step, oversubscription, not a baseline."""
    host = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = host
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
                q = float(fh.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                per = float(fh.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    usable = min(host, aff, int(quota) if quota else host)
    # the GPU boxes also state the per-process CPU share in OMP_NUM_THREADS (16)
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        usable = min(usable, int(share))
    return {"host_logical_cpus": host, "affinity_cpus": aff,
            "cgroup_cpu_quota": round(quota, 2) if quota else None,
            "omp_num_threads": int(share) if share.isdigit() else None, "usable_cpus": max(1, usable)}


def cpu_baseline(cfg, params, spk, B: int, T: int, seconds: float, threads: int):
    """The reference's CPU path -- its module graph on torch fp32 CPU (oneDNN
    convolutions), restated in oracle/torch_cpu.py and pinned to the reference
    fixtures by tests/test_torch_cpu_baseline.py -- on a bounded sample of the
    same workload: the whole (B, 1, T) encode+decode step, repeated for about
    ``seconds`` of wall time (at least twice) on ``threads`` intra-op threads,
    then the same step on ONE thread (at least twice, about seconds / 2), with
    the host's CPU model and load before and after, so that box-to-box swings of
    the shared GPU hosts can be told apart from the code's."""
    import torch
    from oracle.torch_cpu import TorchCPURave
    before = host_info()
    m = TorchCPURave(cfg, params, spk)
    x = torch.from_numpy(synth_batch(B, T, 0))

    def timed(nthreads, secs):
        torch.set_num_threads(nthreads)
        m.forward(x)   # warm-up (oneDNN primitive creation)
        n, t0 = 0, time.perf_counter()
        while True:
            m.forward(x)
            n += 1
            el = time.perf_counter() - t0
            if el >= secs and n >= 2:
                return n, el

    n, el = timed(threads, seconds)
    n1, el1 = timed(1, seconds / 2)
    # every CPU this process may use (BASELINE.md's plan: all host cores, the
    # count stated): the affinity mask and cgroup quota bound it on a shared host
    cpus = usable_cpus()
    allc = cpus["usable_cpus"]
    load_all = host_info()["loadavg_1min"]
    if allc != threads:
        na, ela = timed(allc, seconds / 2)
    else:                                    # the main figure already used them all
        na, ela = n, el
    after = host_info()
    torch.set_num_threads(threads)
    return {"value": round(n * B * T / el, 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "ms_per_step": round(1e3 * el / n, 2),
            "one_thread": {"value": round(n1 * B * T / el1, 1), "ms_per_step": round(1e3 * el1 / n1, 2),
                           "steps": n1},
            "all_host_cores": {"threads": allc, "value": round(na * B * T / ela, 1),
                               "ms_per_step": round(1e3 * ela / na, 2), "steps": na,
                               "loadavg_1min_before": load_all, **cpus,
                               "note": "all CPUs the process may use (affinity and cgroup quota of the shared "
                                       "host); the host's logical CPUs beyond the quota are other tenants'"},
            "host": {"cpu_model": before["cpu_model"], "os_cpu_count": before["os_cpu_count"],
                     "loadavg_1min_before": before["loadavg_1min"], "loadavg_1min_after": after["loadavg_1min"]},
            "sample": f"{n} x v2 encode+decode of the bench step ({B} x {T} samples): the reference's "
                      f"module graph on torch {torch.__version__} fp32 CPU (oneDNN), {el:.1f} s wall, "
                      f"torch.set_num_threads({threads}); then {n1} steps on 1 thread ({el1:.1f} s); all usable CPUs: "
                      f"{allc} ({na} steps, {ela:.1f} s)"}


def _pinned(name: str, precision: str):
    """(tuning list or None, its source) of a side config's committed launch choices."""
    path = os.path.join(REPO, "profiles", "tuning", f"{name}_{precision}.json")
    if not os.path.exists(path):
        return None, "autotuned at plan build"
    with open(path) as fh:
        return json.load(fh), os.path.relpath(path, REPO)


def _save_pinned(name: str, precision: str, model) -> None:
    path = os.path.join(REPO, "profiles", "tuning", f"{name}_{precision}.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        json.dump(model.tuning(), fh, indent=0)


def side_configs(a, dev) -> dict:
    """BASELINE configs 3, 4 and 5 on this GPU (N = 1 only), beside the config-2
    headline, in the headline's arithmetic (f32_bf3) and in ``auto``; every
    number from the same process as the headline:

    * C3 -- v2 causal streaming, 2048-sample blocks, B = 1 (one nn~ stream):
      host call -> synchronize latency of each block, median and p99 over
      ``a.c3_blocks`` blocks after 8 warm-up blocks, each block a replayed
      hipGraph, for decode and for encode+decode; kernel launches per block;
    * C4 -- discrete encode_codes -> decode_codes of the per-GPU shard of 64
      clips over 8 GPUs (8 x 65536), ms per shard (the RVQ-index all-gather is
      an identity at N = 1);
    * C5 -- v3 Snake + noise decode of the per-GPU shard of 128 (z 16 x 320 x 64
      -> 16 x 65536), noise drawn on the device, ms per shard.

    Synthetic inputs, seeded random-init weights.  Launch choices are pinned by
    profiles/tuning/{c3,c4,c5}_<precision>.json where committed."""
    import torch
    from rave_amd import config as rcfg
    from rave_amd.model import DECODE, DECODE_CODES, ENCODE_CODES, RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker

    def sync_ms(fn, steps, warmup):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    out = {"note": "N = 1, synthetic inputs, random-init weights; C3 per-block latency = host call -> "
                   "synchronize of one replayed block graph (plus its two staging copies)"}
    for prec in ("f32_bf3", "auto"):
        res = {}
        # ---- C3
        cfg = rcfg.causal()
        tun, src = _pinned("c3", prec)
        m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=prec, tuning=tun)
        blk, warm, nb = 2048, 8, a.c3_blocks
        gen = torch.Generator().manual_seed(0)
        z = torch.randn(warm + nb, 1, cfg.dec_in, blk // cfg.hop, generator=gen).to(dev)
        x = (0.2 * torch.randn(warm + nb, 1, 1, blk, generator=gen)).to(dev)
        s = StreamingRAVE(m, batch=1, block=blk, graph=True)
        c3 = {"workload": "v2 causal streaming, 2048-sample blocks, B = 1 (BASELINE configs[2])",
              "tuning": src, "launches_per_block": {"encode": s.launches("encode"), "decode": s.launches("decode")}}
        for name, fn in (("decode", lambda i: s.decode(z[i])), ("encode_decode", lambda i: s.forward(x[i]))):
            s.reset()
            lat = []
            for i in range(warm + nb):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                fn(i)
                torch.cuda.synchronize()
                if i >= warm:
                    lat.append((time.perf_counter() - t0) * 1e3)
            lat = np.array(lat)
            c3[name] = {"median_ms": round(float(np.median(lat)), 4), "p99_ms": round(float(np.percentile(lat, 99)), 4),
                        "x_realtime_at_p99": round(blk / SR * 1e3 / float(np.percentile(lat, 99)), 1)}
        if a.save_tuning:
            _save_pinned("c3", prec, m)
        del s, m
        res["c3"] = c3
        # ---- C4
        cfg = rcfg.discrete()
        tun, src = _pinned("c4", prec)
        m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=prec, tuning=tun)
        B4, T4 = 8, 65536
        x4 = (0.2 * torch.randn(B4, 1, T4, generator=torch.Generator().manual_seed(0))).to(dev)
        ms = sync_ms(lambda: m.decode_codes(m.encode_codes(x4)), a.steps, max(2, a.warmup))
        nl = len(m.ops(ENCODE_CODES, B4, T4)) + len(m.ops(DECODE_CODES, B4, T4 // cfg.hop))
        res["c4"] = {"workload": f"discrete encode_codes -> decode_codes, {B4} x {T4} (BASELINE configs[3], per-GPU "
                                 "shard of 64)", "tuning": src, "ms_per_shard": round(ms, 4),
                     "samples_per_s": round(B4 * T4 / ms * 1e3, 1), "launches": nl}
        if a.save_tuning:
            _save_pinned("c4", prec, m)
        del m
        # ---- C5
        cfg = rcfg.v3_noise()
        tun, src = _pinned("c5", prec)
        m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=prec, tuning=tun)
        B5, F5 = 16, 64
        z5 = torch.randn(B5, cfg.dec_in, F5, generator=torch.Generator().manual_seed(0)).to(dev)
        ms = sync_ms(lambda: m.decode(z5), a.steps, max(2, a.warmup))
        res["c5"] = {"workload": f"v3 Snake + noise decode, z ({B5}, {cfg.dec_in}, {F5}) -> ({B5}, 1, {F5 * cfg.hop}) "
                                 "(BASELINE configs[4], per-GPU shard of 128)", "tuning": src,
                     "ms_per_shard": round(ms, 4), "samples_per_s": round(B5 * F5 * cfg.hop / ms * 1e3, 1),
                     "launches": len(m.ops(DECODE, B5, F5))}
        if a.save_tuning:
            _save_pinned("c5", prec, m)
        del m
        out[prec] = res
        log(f"configs [{prec}]: {json.dumps(res)}")
    return out


DTYPE = {"f32": "fp32 (exact fp32 MFMA v_mfma_f32_32x32x2_f32)",
         "f32_tuned": "fp32 (exact fp32 MFMA v_mfma_f32_32x32x2_f32 on every op; per conv the faster of the "
                      "register-staged kernel and the LDS-DMA ring kernel, launch configurations and "
                      "fused/unfused units autotuned)",
         "f32_bf3": "fp32 (per conv / fused unit the faster of exact-fp32 MFMA and fp32 on the bf16 matrix "
                    "cores: operands split exactly into 3 bf16 parts (24 significand bits), 6 of the 9 cross "
                    "products (the 3 dropped are each < 2^-25 |a b|), fp32 accumulate; edges exact-fp32 MFMA)",
         "split16": "fp32 I/O, split-f16 GEMMs (3 f16 MFMA passes hi*hi+hi*lo+lo*hi on ~22-bit operands, "
                    "fp32 accumulate)",
         "auto": "fp32 I/O; per op the faster of exact-fp32 MFMA and split-f16 GEMMs (3 f16 MFMA passes on "
                 "~22-bit operands, fp32 accumulate)"}


def pipelined(a, cfg, params, spk, precision, model, x, dev):
    """Serving-pipeline throughput beside the headline: ``a.pipeline``
    independent steps in flight, step i on HIP stream i % depth with its own
    engine instance (plans and workspaces are per instance; same tuning, same
    kernels, the same 16-clip encode+decode per step).  Kernels of one step
    fill the CUs another step's launches leave idle (prologues, epilogues,
    one-round grids).  Not the headline ``value``."""
    import torch
    from rave_amd.model import RAVE
    depth = a.pipeline
    models = [model] + [RAVE(cfg, params, spk, device=dev, precision=precision, tuning=model.tuning())
                        for _ in range(depth - 1)]
    streams = [torch.cuda.Stream(dev) for _ in range(depth)]
    B, T = x.shape[0], x.shape[-1]

    def run(k):
        ev = torch.cuda.Event()
        ev.record()
        for s in streams:
            s.wait_event(ev)
        last = [None] * depth          # every stream's last output
        for i in range(k):
            with torch.cuda.stream(streams[i % depth]):
                m = models[i % depth]
                last[i % depth] = m.decode(m.encode(x))
        for s in streams:
            torch.cuda.current_stream(dev).wait_stream(s)
        return [y for y in last if y is not None]

    run(depth * max(1, a.warmup))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ys = run(a.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    # every stream's output finite, and no cooperative-unit give-up in any step
    # (the engine's status words are sticky until read: rave_model_check)
    if not all(bool(torch.isfinite(y).all()) for y in ys):
        raise RuntimeError("non-finite output (pipelined)")
    for m in models:
        m.check()
    v = B * T * a.steps / el
    return {"streams": depth, "value": round(v, 1), "ms_per_step": round(1e3 * el / a.steps, 4),
            "x_realtime": round(v / SR, 1),
            "note": f"{depth} independent {B}-clip encode+decode steps in flight on {depth} HIP streams "
                    "(one engine instance each); reported beside, not as, the headline"}


def timed_region(step, steps: int, warmup: int, world: int, sync, device):
    """The contract's timed region: ``warmup`` untimed steps, then exactly
    ``steps`` steps bracketed by sync + barrier on both sides; the elapsed time
    is the MAX over ranks (all-reduced, so every rank returns it).  Returns
    (seconds, the last step's output).  ``sync`` is torch.cuda.synchronize on
    the GPU; the gloo tests pass a no-op and ``device`` cpu
    (tests/test_distributed_gloo.py)."""
    import torch
    import torch.distributed as dist
    for _ in range(warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    y = None
    for _ in range(steps):
        y = step()
    sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, y


def run_mode(a, cfg, params, spk, precision, x, dev, world, rank, log_ops):
    """Build the model in one arithmetic mode, time K steps (barrier +
    synchronize on both sides, max over ranks) and, unless --no-profile, the
    per-op HIP-event pass.  Returns (result dict, last output)."""
    import torch
    import torch.distributed as dist
    from rave_amd.distributed import ShardedRunner
    from rave_amd.model import RAVE

    B, T = x.shape[0], x.shape[-1]
    # the plan's launch choices: pinned by the committed tuning file of this
    # workload and arithmetic mode (profiles/tuning/), so every box runs the same
    # arithmetic mix and kernels; --retune times them afresh at plan build
    tuning, src = None, "autotuned at plan build"
    path = a.tuning_in if (a.tuning_in and precision == a.precision) else None
    if path is None and not a.retune and os.path.exists(tuning_path(cfg.name, B, T, precision)):
        path = tuning_path(cfg.name, B, T, precision)
    if path:
        with open(path) as fh:
            tuning = json.load(fh)
        src = os.path.relpath(path, REPO)
    model = RAVE(cfg, params, spk, device=dev, precision=precision, tuning=tuning)
    Fz = T // cfg.hop
    runner = ShardedRunner(model, shard_sizes=[B] * world)   # encode -> RCCL all-gather of latents -> decode

    def step():
        return runner.step(x)[1]

    from rave_amd.model import DECODE, ENCODE
    plans = ((ENCODE, T), (DECODE, Fz))
    ops = {w: model.ops(w, B, t) for w, t in plans}          # builds (and autotunes) both plans
    eff = model.tuning()
    if a.tuning_out and rank == 0 and precision == a.precision:
        with open(a.tuning_out, "w") as fh:
            json.dump(eff, fh)
    if a.save_tuning and rank == 0:
        os.makedirs(os.path.dirname(tuning_path(cfg.name, B, T, precision)), exist_ok=True)
        with open(tuning_path(cfg.name, B, T, precision), "w") as fh:
            json.dump(eff, fh, indent=0)
    tuning_info = {"source": src, "sha16": tuning_hash(eff), "entries": len(eff),
                   "retimed": (len(eff) - len(tuning)) if tuning is not None else len(eff)}
    el, y = timed_region(step, a.steps, a.warmup, world, torch.cuda.synchronize, dev)
    if a.timing_only_variant:     # A/B of a timing-only kernel variant: results are not meaningful
        gather_check = {"checked": False, "reason": "timing-only kernel variant"}
    else:
        if not torch.isfinite(y).all():
            raise RuntimeError("non-finite output")
        model.check()     # a cooperative-unit give-up in any timed step is an error, not a number
        # the exchange checked end to end, outside the timed region: every rank's
        # rows of the gathered latents against that rank's own (raises on mismatch)
        gather_check = runner.verify(x)
    value = world * B * T * a.steps / el
    res = {"value": round(value, 1), "ms_per_step": round(1e3 * el / a.steps, 4),
           "x_realtime": round(value / SR, 1), "dtype": DTYPE[precision], "tuning": tuning_info,
           "gather_check": gather_check}
    if a.pipeline > 1 and world == 1 and precision == a.precision:
        res["pipelined"] = pipelined(a, cfg, params, spk, precision, model, x, dev)
    launches = {}
    for w, _ in plans:
        for o in ops[w]:
            fam = op_family(o["kind"], o["precision"])
            if fam in FAMILIES:
                launches[fam] = launches.get(fam, 0) + 1
    res["gemm_launches_by_family"] = launches
    if a.no_profile:
        return res, y

    # ---------------------------------------------------------- roofline (HIP events per op)
    # Per-op timing over a second pass of the same K steps: the events ride
    # inside the kernels' own dispatch packets (hipExtLaunchKernelGGL on the
    # plan's stream, no marker packets, no host syncs).  Kept out of the timed
    # pass above, whose wall time the event bookkeeping would stretch (~15 %).
    for w, t in plans:
        model.profile(w, B, t, a.steps)
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    times = {}
    for w, t in plans:
        tm, nr = model.op_times(w, B, t)
        model.profile(w, B, t, 0)
        if nr != a.steps:
            raise RuntimeError(f"profiled {nr} runs of plan {w}, expected {a.steps}")
        times[w] = tm / a.steps
    te, td = times[ENCODE], times[DECODE]
    rows = []
    fams: dict = {}
    for w, _ in plans:
        for o, ms in zip(ops[w], times[w]):
            lab, fl, nb = o["label"], o["flops"], o["bytes"]
            fam = op_family(o["kind"], o["precision"])
            rows.append((lab, fam, fl, nb, ms))
            if fam in FAMILIES:
                f = fams.setdefault(fam, [0, 0.0, 0.0, 0.0])
                f[0] += 1
                f[1] += fl
                f[2] += nb
                f[3] += float(ms)
    traffic = traffic_per_launch(cfg.name, B, T, precision)

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
    res["roofline"] = {
        "bound": d["bound"], "achieved": d["achieved"], "peak": d["peak"], "unit": d["unit"],
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
    if log_ops:
        log(f"[{precision}] {'op':58s} {'family':14s} {'GFLOP':>8s} {'MB':>7s} {'ms':>8s} {'TFLOP/s':>8s} "
            f"{'GB/s':>7s}")
        for lab, fam, fl, nb, ms in rows:
            ms_ = max(ms, 1e-9)
            log(f"[{precision}] {lab[-58:]:58s} {fam:14s} {fl / 1e9:8.3f} {nb / 1e6:7.2f} {ms:8.4f} "
                f"{fl / ms_ / 1e9:8.2f} {nb / ms_ / 1e6:7.0f}")
    return res, y


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv) -> int:
    """``--gpus N`` without a torch.distributed environment: start N rank
    processes (one per GPU) under torch.distributed.run on 127.0.0.1 as a CHILD
    process -- this parent never touches the GPU and never execs -- and return
    its exit code.  Rank 0's JSON line reaches stdout unchanged."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    log(f"bench: launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd, env=env)


def dry_run(a, world: int, rank: int) -> None:
    """``--dry-run``: the launcher and rank bookkeeping without a GPU -- gloo
    process group, barrier, max-over-ranks of a dummy timing -- and the same
    rank-0 JSON line skeleton (tests/test_bench_launcher.py)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
        t = torch.tensor([float(rank)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        seen = dist.get_world_size()
    else:
        seen = 1
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "samples/s", "n_gpus": a.gpus,
                          "ranks_seen": seen, "steps": a.steps, "warmup": a.warmup, "dry_run": True}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE in the environment bench.py launches them")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the launcher / process group on gloo and print a skeleton line")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="clips per GPU")
    ap.add_argument("--samples", type=int, default=65536, help="samples per clip")
    ap.add_argument("--config", default="v2")
    ap.add_argument("--precision", default="f32_bf3", choices=["f32", "f32_tuned", "f32_bf3", "split16", "auto"],
                    help="conv/unit GEMM arithmetic of the headline (include/rave_amd.h RAVE_PREC_*). "
                         "Default f32_bf3: fp32 on every op (exact fp32 MFMA, or for fused units bf16x3 with "
                         "an exact operand split), launch choices pinned; f32_tuned = exact fp32 MFMA on "
                         "every op; auto = per op the faster of exact fp32 and split-f16")
    ap.add_argument("--no-f32", "--no-secondary", dest="no_f32", action="store_true",
                    help="skip the arithmetic modes that ride along the headline (exact fp32 and auto "
                         "beside f32_bf3; auto beside f32_tuned; exact fp32 beside auto)")
    ap.add_argument("--tuning-in", help="JSON of RAVE.tuning() to reuse (no timing runs at plan build)")
    ap.add_argument("--tuning-out", help="write RAVE.tuning() here after the plans are built")
    ap.add_argument("--retune", action="store_true",
                    help="ignore the committed profiles/tuning/ files: time every launch choice at plan build")
    ap.add_argument("--timing-only-variant", action="store_true",
                    help="A/B runs of a timing-only kernel variant library (RAVE_AMD_LIB_VARIANT): skip the "
                         "output checks; refused for the product library")
    ap.add_argument("--save-tuning", action="store_true",
                    help="write each mode's effective launch choices to profiles/tuning/ (to pin them)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="torch CPU threads of the baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip BASELINE configs 3-5 (C3 streaming latency, C4 / C5 shards) beside the headline")
    ap.add_argument("--c3-blocks", type=int, default=64, help="timed C3 blocks per measurement")
    ap.add_argument("--pipeline", type=int, default=3,
                    help="also time this many independent steps in flight on as many streams (N=1 only; "
                         "reported as 'pipelined' beside the headline; 1 = off)")
    a = ap.parse_args()
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if a.timing_only_variant and not os.environ.get("RAVE_AMD_LIB_VARIANT"):
        ap.error("--timing-only-variant is for RAVE_AMD_LIB_VARIANT libraries only")
    if "WORLD_SIZE" not in os.environ:
        if a.gpus > 1:
            sys.exit(launch_ranks(a.gpus, sys.argv[1:]))
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if world != a.gpus:
            log(f"bench: WORLD_SIZE={world} but --gpus {a.gpus}; refusing to report a mislabelled run")
            sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_run:
        dry_run(a, world, rank)
        return

    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")

    from rave_amd import config as rcfg
    from rave_amd.weights import init_params, init_speaker

    cfg = rcfg.get_config(a.config)
    params = init_params(cfg, seed=0)
    spk = init_speaker(cfg, seed=0)
    B, T = a.batch, a.samples
    x = torch.from_numpy(synth_batch(B, T, 1000 * rank)).to(dev)

    head, y_head = run_mode(a, cfg, params, spk, a.precision, x, dev, world, rank, rank == 0)
    exact = None
    fast = None
    if a.precision not in ("f32", "f32_tuned") and not a.no_f32:
        # exact fp32 MFMA on every op, with the same launch-configuration autotuning as the headline
        exact, y_f32 = run_mode(a, cfg, params, spk, "f32_tuned", x, dev, world, rank, rank == 0)
        # the same input through both arithmetic modes (north star: <= 1e-4 max-abs)
        exact["headline_vs_f32_max_abs"] = float((y_head - y_f32).abs().max())
        del y_f32
    if a.precision not in ("auto", "split16") and not a.no_f32:
        # the fastest mixed mode (per op exact fp32 or split-f16, ~22-bit operands),
        # its error against the headline on the same input
        fast, y_fast = run_mode(a, cfg, params, spk, "auto", x, dev, world, rank, rank == 0)
        fast["vs_headline_max_abs"] = float((y_head - y_fast).abs().max())
        fast["precision"] = "auto"
        del y_fast

    side = None
    if world == 1 and not a.no_configs:
        side = side_configs(a, dev)

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(cfg, params, spk, B, T, a.cpu_seconds, a.cpu_threads)

    if rank == 0:
        out = {
            "metric": METRIC, "value": head["value"], "unit": "samples/s", "n_gpus": world,
            "ranks_seen": dist.get_world_size() if world > 1 else 1,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": head["ms_per_step"],
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": head["dtype"],
            "precision": a.precision,
            "data": "synthetic (440 Hz sine + N(0,0.1) noise; seeded random-init v2 weights)",
            "config": {"workload": f"{cfg.name} non-causal encode+decode, {B} x {T} samples per GPU "
                                   "(BASELINE configs[1])",
                       "global_batch": world * B, "samples_per_clip": T,
                       "parallelism": f"dp{world} (batch shards, RCCL all-gather of latents)"},
            "x_realtime": head["x_realtime"],
            "per_gpu_samples_per_s": round(head["value"] / world, 1),
            "gemm_launches_by_family": head["gemm_launches_by_family"],
            "tuning": head["tuning"],
            "gather_check": head["gather_check"],
            "roofline": head.get("roofline"),
            "pipelined": head.get("pipelined"),
            "f32_exact": exact,
            "split16_auto": fast,
            "configs": side,
            "cpu_baseline": cpu,
        }
        for side in (exact, fast):                # keep the second mode's roofline compact
            if side and side.get("roofline"):
                r = side["roofline"]
                side["roofline"] = {k: r[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                      "kernel", "all_gemm_ops")}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
