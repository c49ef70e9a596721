#!/usr/bin/env python3
"""Probe: one bench step (16 x 65536 v2 encode+decode) with the batch split
into P independent shards on P HIP streams (one engine instance per shard),
against the same step on one stream.  Prints ms per step for P = 1, 2, 4.
Measurement only (tools/, not the product path)."""
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from bench import synth_batch  # noqa: E402
from rave_amd import config as rcfg  # noqa: E402
from rave_amd.model import RAVE  # noqa: E402
from rave_amd.weights import init_params, init_speaker  # noqa: E402


def main():
    steps, warm = 20, 5
    dev = torch.device("cuda:0")
    cfg = rcfg.get_config("v2")
    params = init_params(cfg, seed=0)
    spk = init_speaker(cfg, seed=0)
    B, T = 16, 65536
    x = torch.from_numpy(synth_batch(B, T, 0)).to(dev)
    out = {}
    ref = None
    for P in (1, 2, 4):
        sb = B // P
        models = [RAVE(cfg, params, spk, device=dev, precision="auto") for _ in range(P)]
        streams = [torch.cuda.Stream(dev) for _ in range(P)]
        ys = [None] * P

        def step():
            ev = torch.cuda.Event()
            ev.record()
            for i in range(P):
                streams[i].wait_event(ev)
                with torch.cuda.stream(streams[i]):
                    m = models[i]
                    ys[i] = m.decode(m.encode(x[i * sb:(i + 1) * sb]))
            for s in streams:
                torch.cuda.current_stream(dev).wait_stream(s)

        for _ in range(warm):
            step()
        torch.cuda.synchronize()
        best = 1e9
        for _rep in range(3):
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / steps * 1e3)
        y = torch.cat(ys, 0)
        if ref is None:
            ref = y.clone()
        out[P] = {"ms_per_step": round(best, 4), "max_abs_vs_P1": float((y - ref).abs().max())}
        print(f"P={P}: {out[P]}", file=sys.stderr, flush=True)
        del models
    print(json.dumps(out))


if __name__ == "__main__":
    main()
