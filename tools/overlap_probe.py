#!/usr/bin/env python3
"""Throughput of independent full-batch passes overlapped on two HIP streams
(e.g. step k+1's encode beside step k's decode in a serving loop) against the
same passes back to back on one stream.  Each launch keeps its full grid; the
second stream's workgroups can only use what the first leaves idle (tails,
partially filled CUs).

    python tools/overlap_probe.py [--batch 16] [--iters 20]
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
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    cfg = rcfg.v2()
    params, spk = init_params(cfg, 0), init_speaker(cfg, 0)
    dev = torch.device("cuda")
    B, T = a.batch, 65536
    ma = RAVE(cfg, params, spk, device=dev, precision="auto")
    mb = RAVE(cfg, params, spk, device=dev, precision="auto", tuning=ma.tuning())
    xs = [0.1 * torch.randn(B, 1, T, device=dev) for _ in range(2)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def serial():
        for _ in range(a.iters):
            ma.forward(xs[0])
            mb.forward(xs[1])

    def overlapped():
        ev = torch.cuda.Event()
        ev.record()
        for m, x, st in ((ma, xs[0], s1), (mb, xs[1], s2)):
            st.wait_event(ev)
            with torch.cuda.stream(st):
                for _ in range(a.iters):
                    m.forward(x)
        for st in (s1, s2):
            torch.cuda.current_stream().wait_stream(st)

    for name, fn in (("serial, 1 stream", serial), ("overlapped, 2 streams", overlapped)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / (2 * a.iters)
        print(f"{name:24s} {ms:7.3f} ms per {B}x{T} forward", flush=True)


if __name__ == "__main__":
    main()
