#!/usr/bin/env python3
"""Single-GPU measurements of BASELINE.json configs 3, 4 and 5 (bench.py is the
config-2 line).  SURVEY.md section 8d:

* C3 -- v2 causal streaming (cached_conv semantics), 2048-sample blocks, B=1:
  per-block latency (host call -> synchronize, median / p99 over >= 64 blocks
  after warm-up) of decode and of encode+decode, and the steady-state
  throughput of back-to-back blocks (no per-block synchronize).
* C4 -- discrete encode -> RVQ -> decode (encode_codes + decode_codes), the
  per-GPU shard of batch 64 over 8 GPUs: 8 x 65536 samples.
* C5 -- v3 Snake + noise decode, the per-GPU shard of batch 128 over 8 GPUs:
  z (16, 320, 64) -> (16, 1, 65536), noise drawn on the device.

Synthetic inputs and random-init weights (rave_amd.weights), as bench.py.
Prints one JSON object; the reference CPU numbers these compare with are in
BASELINE.md (measured in the build container, 8 threads).

    python tools/configs_bench.py [--precision auto] [--only c3,c4,c5]

C4 and C5 run through rave_amd.distributed.ShardedRunner; launched with
``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1
tools/configs_bench.py --only c4,c5`` each rank takes one shard (weak scaling)
and the numbers are whole-job (max over ranks), as in bench.py.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rave_amd import config as rcfg  # noqa: E402
from rave_amd.distributed import ShardedRunner, world  # noqa: E402
from rave_amd.model import RAVE  # noqa: E402
from rave_amd.weights import init_params, init_speaker  # noqa: E402

SR = 48000


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def timed_steps(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def c3(precision, blocks, warmup, dev):
    from rave_amd.streaming import StreamingRAVE
    cfg = rcfg.causal()
    m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=precision)
    blk = 2048
    Fz = blk // cfg.hop
    n = warmup + blocks
    gen = torch.Generator().manual_seed(0)
    z = torch.randn(n, 1, cfg.dec_in, Fz, generator=gen).to(dev)
    x = (0.2 * torch.randn(n, 1, 1, blk, generator=gen)).to(dev)
    out = {"workload": "v2 --config causal streaming, 2048-sample blocks, B=1 (BASELINE configs[2])",
           "block_samples": blk, "blocks_timed": blocks}
    runs = []
    for graph in (True, False):
        s = StreamingRAVE(m, batch=1, block=blk, graph=graph)
        out["decode_delay_samples"] = s.decode_delay
        tag = "" if graph else "_eager"
        runs += [("decode" + tag, s, (lambda s: lambda i: s.decode(z[i]))(s)),
                 ("encode_decode" + tag, s, (lambda s: lambda i: s.forward(x[i]))(s))]
    out["note"] = "default: each block replays a captured hipGraph (RAVE_STREAM_GRAPH); *_eager: plan replay"
    for name, s, fn in runs:
        s.reset()
        lat = []
        for i in range(n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn(i)
            torch.cuda.synchronize()
            if i >= warmup:
                lat.append(time.perf_counter() - t0)
        lat = np.array(lat) * 1e3
        med = float(np.median(lat))
        # back-to-back blocks, one synchronize at the end (a host that keeps the queue fed)
        s.reset()
        for i in range(warmup):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(warmup, n):
            fn(i)
        torch.cuda.synchronize()
        thr_ms = (time.perf_counter() - t0) / blocks * 1e3
        out[name] = {"latency_ms_median": round(med, 4), "latency_ms_p99": round(float(np.percentile(lat, 99)), 4),
                     "x_realtime_at_median_latency": round(blk / SR * 1e3 / med, 1),
                     "pipelined_ms_per_block": round(thr_ms, 4),
                     "pipelined_x_realtime": round(blk / SR * 1e3 / thr_ms, 1)}
        log(f"C3 {name}: {out[name]}")
    return out


def sharded_steps(fn, steps, warmup):
    """bench.py's contract (bench.timed_region, the same code): barrier +
    synchronize around exactly ``steps`` steps, the max over ranks."""
    from bench import timed_region
    rank, size = world()
    el, _ = timed_region(fn, steps, warmup, size, torch.cuda.synchronize, torch.device("cuda"))
    return el / steps


def c4(precision, steps, warmup, dev, B=8, T=65536):
    """Per-GPU shard of 64: encode_codes -> all-gather of the indices (RCCL,
    int16 on the wire) -> decode_codes (rave_amd.distributed, mode "codes")."""
    rank, size = world()
    cfg = rcfg.discrete()
    m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=precision)
    x = (0.2 * torch.randn(B, 1, T, generator=torch.Generator().manual_seed(rank))).to(dev)
    t_enc = timed_steps(lambda: m.encode_codes(x), steps, warmup)
    idx = m.encode_codes(x)
    t_dec = timed_steps(lambda: m.decode_codes(idx), steps, warmup)
    runner = ShardedRunner(m, mode="codes")
    t = sharded_steps(lambda: runner.step(x), steps, warmup)
    out = {"workload": f"discrete encode -> RVQ(16x1024) -> all-gather indices -> decode, {B} x {T} per GPU "
                       "(BASELINE configs[3] per-GPU shard of 64)", "n_gpus": size,
           "ms_per_step": round(t * 1e3, 4), "encode_codes_ms": round(t_enc * 1e3, 4),
           "decode_codes_ms": round(t_dec * 1e3, 4),
           "samples_per_s": round(size * B * T / t, 1), "x_realtime_aggregate": round(size * B * T / t / SR, 1)}
    log(f"C4: {out}")
    return out


def c5(precision, steps, warmup, dev, B=16, Fz=64):
    """Per-GPU shard of 128: decode of the local latents, no exchange
    (rave_amd.distributed, mode "decode")."""
    rank, size = world()
    cfg = rcfg.v3_noise()
    m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=precision)
    z = torch.randn(B, cfg.dec_in, Fz, generator=torch.Generator().manual_seed(rank)).to(dev)
    runner = ShardedRunner(m, mode="decode")
    t = sharded_steps(lambda: runner.step(z), steps, warmup)
    T = Fz * cfg.hop
    out = {"workload": f"v3 Snake + noise decode, z ({B}, {cfg.dec_in}, {Fz}) -> ({B}, 1, {T}) per GPU "
                       "(BASELINE configs[4] per-GPU shard of 128), device-drawn noise", "n_gpus": size,
           "ms_per_step": round(t * 1e3, 4), "samples_per_s": round(size * B * T / t, 1),
           "x_realtime_aggregate": round(size * B * T / t / SR, 1)}
    log(f"C5: {out}")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="auto", choices=["f32", "f32_tuned", "f32_bf3", "split16", "auto"])
    ap.add_argument("--only", default="c3,c4,c5")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--blocks", type=int, default=64)
    a = ap.parse_args()
    size = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if size > 1:     # torch.distributed.run, one process per GPU, RCCL
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    which = set(a.only.split(","))
    res = {"precision": a.precision, "device": torch.cuda.get_device_name(local), "data": "synthetic",
           "weights": "random-init (rave_amd.weights)", "n_gpus": size}
    if "c3" in which and size == 1:      # one stream per nn~ instance: not sharded
        res["c3"] = c3(a.precision, a.blocks, 8, dev)
    if "c4" in which:
        res["c4"] = c4(a.precision, a.steps, a.warmup, dev)
    if "c5" in which:
        res["c5"] = c5(a.precision, a.steps, a.warmup, dev)
    if world()[0] == 0:
        print(json.dumps(res))
    if size > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
