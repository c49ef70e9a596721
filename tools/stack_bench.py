#!/usr/bin/env python3
"""Time rave_residual_stack against the same three units run one by one
(the unit kernel of the same arithmetic) at the v2 bench sizes:

    python tools/stack_bench.py [--iters 50] [--precision split16|bf16x3]

With RAVE_AMD_DIAG_LIB=1 (the -DRAVE_STAMPS build, csrc/Makefile `diag`) it also
prints the per-workgroup clock stamps of one stack launch (segments: window
staging, unit 0, unit 1, unit 2, stores) and of the units.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rave_amd import _native as N  # noqa: E402
from tools.layer_bench import STAMPS, stamp_report  # noqa: E402

SIZES = {64: 4096, 128: 1024}     # channels: samples per clip at that stage of v2 (B = 16)


def timeit(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--precision", default="split16", choices=["split16", "bf16x3"])
    a = ap.parse_args()
    prec = N.PRECISION[a.precision]
    dev = torch.device("cuda")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(0)
    for Cc, T in SIZES.items():
        B = a.batch
        x = torch.randn(B, Cc, T, device=dev)
        y = torch.empty_like(x)
        tmp = [torch.empty_like(x) for _ in range(2)]
        sa = N.StackArgs(channels=Cc, batch=B, t_len=T, act=N.ACT["leaky"], leaky_slope=0.2, precision=prec,
                         x=x.data_ptr(), x_sb=Cc * T, x_sc=T, y=y.data_ptr(), y_sb=Cc * T, y_sc=T)
        keep, units = [], []
        for u, d in enumerate((1, 3, 9)):
            w1 = (rng.standard_normal((Cc, Cc, 3)) / np.sqrt(3 * Cc)).astype(np.float32)
            w2 = (rng.standard_normal((Cc, Cc, 1)) / np.sqrt(Cc)).astype(np.float32)
            pw = torch.from_numpy(N.pack_unit_weight(w1, w2, Cc, precision=prec)).to(dev)
            b1, b2 = torch.randn(Cc, device=dev) * 0.1, torch.randn(Cc, device=dev) * 0.1
            keep += [pw, b1, b2]
            setattr(sa, f"dilation{u}", d)
            setattr(sa, f"pad_left{u}", d)
            setattr(sa, f"weight{u}", pw.data_ptr())
            setattr(sa, f"bias1{u}", b1.data_ptr())
            setattr(sa, f"bias2{u}", b2.data_ptr())
            src = x if u == 0 else tmp[(u - 1) % 2]
            dst = y if u == 2 else tmp[u % 2]
            units.append(N.UnitArgs(channels=Cc, batch=B, t_len=T, dilation=d, pad_left=d, act=N.ACT["leaky"],
                                    leaky_slope=0.2, precision=prec, x=src.data_ptr(), x_sb=Cc * T,
                                    x_sc=T, y=dst.data_ptr(), y_sb=Cc * T, y_sc=T, weight=pw.data_ptr(),
                                    bias1=b1.data_ptr(), bias2=b2.data_ptr()))
        t_stack = timeit(lambda: N.check(N.lib.rave_residual_stack(C.byref(sa), st)), a.iters)
        t_units = timeit(lambda: [N.check(N.lib.rave_residual_unit(C.byref(ua), st)) for ua in units], a.iters)
        print(f"C={Cc:4d} T={T:5d} B={B} {a.precision}: stack {t_stack:7.2f} us   3 units {t_units:7.2f} us",
              flush=True)
        if STAMPS:
            for label, setter, fn in (
                    ("stack", N.lib.rave_diag_stack_stamps, lambda: N.lib.rave_residual_stack(C.byref(sa), st)),
                    ("unit 0", N.lib.rave_diag_unit_stamps, lambda: N.lib.rave_residual_unit(C.byref(units[0]), st))):
                stamps = torch.zeros(8 * 200000, dtype=torch.int64, device=dev)
                N.check(setter(C.c_void_p(stamps.data_ptr())))
                N.check(fn())
                torch.cuda.synchronize()
                print(f"  {label} stamps:", flush=True)
                stamp_report(stamps.view(-1, 8).cpu().numpy())
                N.check(setter(C.c_void_p(0)))


if __name__ == "__main__":
    main()
