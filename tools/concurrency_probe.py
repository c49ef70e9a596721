#!/usr/bin/env python3
"""Does running two half-batch plans concurrently on two HIP streams beat one
full-batch plan?  (Latency-bound launches leave SIMDs idle; a second stream's
kernels can fill them if LDS / VGPR budgets let workgroups co-reside.)

    python tools/concurrency_probe.py [--batch 16] [--iters 20]
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
    ap.add_argument("--precision", default="auto")
    a = ap.parse_args()
    cfg = rcfg.v2()
    params, spk = init_params(cfg, 0), init_speaker(cfg, 0)
    dev = torch.device("cuda")
    B, T = a.batch, 65536
    full = RAVE(cfg, params, spk, device=dev, precision=a.precision)
    halves = [RAVE(cfg, params, spk, device=dev, precision=a.precision) for _ in range(2)]
    x = 0.1 * torch.randn(B, 1, T, device=dev)
    xs = [x[: B // 2].contiguous(), x[B // 2:].contiguous()]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def run_full():
        full.forward(x)

    def run_halves():
        ev = torch.cuda.Event()
        ev.record()
        for m, xi, st in zip(halves, xs, streams):
            st.wait_event(ev)
            with torch.cuda.stream(st):
                m.forward(xi)
        for st in streams:
            torch.cuda.current_stream().wait_stream(st)

    def run_halves_serial():
        for m, xi in zip(halves, xs):
            m.forward(xi)

    for name, fn in (("full B", run_full), ("2 halves, 2 streams", run_halves),
                     ("2 halves, 1 stream", run_halves_serial)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.iters
        print(f"{name:24s} {ms:7.3f} ms per {B}x{T} forward", flush=True)
    y_full = full.forward(x)
    y_h = torch.cat([m.forward(xi) for m, xi in zip(halves, xs)])
    torch.cuda.synchronize()
    print(f"max |full - halves| = {float((y_full - y_h).abs().max()):.3g}")


if __name__ == "__main__":
    main()
