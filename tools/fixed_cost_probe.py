#!/usr/bin/env python3
"""Per-launch fixed cost of the split-f16 conv: a k1 conv with c_out = 512 at
N = 16 x 128 columns (the C=512 layer shape of v2) timed at growing c_in, best
launch configuration per point.  The intercept of time vs K is the cost every
layer pays regardless of its work (dispatch, prologue loads, epilogue, tail);
the slope is the K loop's marginal rate.

    python tools/fixed_cost_probe.py [--iters 50]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import layer_bench as LB  # noqa: E402
from rave_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--cout", type=int, default=512)
    ap.add_argument("--t", type=int, default=128)
    a = ap.parse_args()
    LB.PREC = N.PREC_SPLIT16
    dev = torch.device("cuda")
    # back-to-back dependent launches of a one-workgroup kernel: the stream's
    # own per-launch floor
    t1 = torch.zeros(1, device=dev)
    for _ in range(10):
        t1.add_(1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(1000):
        t1.add_(1)
    e1.record()
    torch.cuda.synchronize()
    print(f"empty-ish launch floor: {e0.elapsed_time(e1):.3f} us per launch (1000 x add_ on 1 element)",
          flush=True)
    pts = []
    for ci in (32, 64, 128, 256, 512, 1024, 2048):
        name = f"k1_{ci}x{a.cout}"
        LB.LAYERS[name] = (ci, a.cout, 1, 1, 1, 0, "leaky", False, a.t)
        ms = LB.run(name, 16, a.iters, dev, "all")
        pts.append((ci, ms * 1e3))
    k = np.array([p[0] for p in pts], float)
    us = np.array([p[1] for p in pts], float)
    slope, icpt = np.polyfit(k, us, 1)
    gflop_per_k = 2.0 * 16 * a.t * a.cout / 1e9
    print(f"fit: t = {icpt:.2f} us + {slope * 1e3:.3f} us per 1000 K "
          f"(marginal {gflop_per_k / (slope * 1e-6) / 1e3:.0f} TFLOP/s)", flush=True)
    for ci, t in pts:
        print(f"  K={ci:5d}  {t:7.2f} us   fit {icpt + slope * ci:7.2f}", flush=True)


if __name__ == "__main__":
    main()
