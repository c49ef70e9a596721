#!/usr/bin/env python3
"""Experiment: the config-2 step (16 x 65536 encode+decode) split into k
sub-batches that run concurrently on k HIP streams (one plan per sub-batch).

    python tools/stream_bench.py [--precision split16] [--splits 1,2,4]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rave_amd import config as rcfg  # noqa: E402
from rave_amd.model import RAVE  # noqa: E402
from rave_amd.weights import init_params, init_speaker  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="split16")
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    cfg = rcfg.v2()
    dev = torch.device("cuda")
    m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=a.precision)
    B, T = 16, 65536
    x = 0.1 * torch.randn(B, 1, T, device=dev)
    for k in [int(v) for v in a.splits.split(",")]:
        streams = [torch.cuda.Stream() for _ in range(k)]
        parts = list(x.chunk(k))
        zs = [None] * k

        def step():
            for i, (s, xp) in enumerate(zip(streams, parts)):
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    m.decode(m.encode(xp))
            for s in streams:
                torch.cuda.current_stream().wait_stream(s)

        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.steps
        print(f"{a.precision} splits={k}: {ms:.3f} ms/step  {B * T / ms / 1e3:.1f} Msamples/s", flush=True)


if __name__ == "__main__":
    main()
