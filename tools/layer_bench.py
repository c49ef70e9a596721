#!/usr/bin/env python3
"""Time single conv layers of the v2 graph in isolation (HIP events), for
kernel tuning and per-layer PMC profiling:

    python tools/layer_bench.py [--layers k3_64,k1_64,...] [--iters 50] [--batch 16]
"""
import argparse
import ctypes as C
import ctypes as C_
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rave_amd import _native as N  # noqa: E402

# name: (c_in, c_out, k, s, d, transposed, act, residual, t_in per clip)
LAYERS = {
    "k3_64": (64, 64, 3, 1, 9, 0, "leaky", False, 4096),
    "k1_64": (64, 64, 1, 1, 1, 0, "leaky", True, 4096),
    "k3_128": (128, 128, 3, 1, 3, 0, "leaky", False, 1024),
    "k1_128": (128, 128, 1, 1, 1, 0, "leaky", True, 1024),
    "k3_256": (256, 256, 3, 1, 3, 0, "leaky", False, 256),
    "k1_256": (256, 256, 1, 1, 1, 0, "leaky", True, 256),
    "k3_512": (512, 512, 3, 1, 3, 0, "leaky", False, 128),
    "k1_512": (512, 512, 1, 1, 1, 0, "leaky", True, 128),
    "down4_64": (64, 128, 8, 4, 1, 0, "leaky", False, 4096),
    "down2_256": (256, 512, 4, 2, 1, 0, "leaky", False, 256),
    "convT2_1024": (1024, 512, 4, 2, 1, 1, "leaky", False, 64),
    "down2_512": (512, 1024, 4, 2, 1, 0, "leaky", False, 128),
    "convT4_128": (128, 64, 8, 4, 1, 1, "leaky", False, 1024),
    "enc_out": (1024, 64, 3, 1, 1, 0, "leaky", False, 64),
    "dec_in": (320, 1024, 3, 1, 1, 0, "none", False, 64),
    "wave": (64, 32, 7, 1, 1, 0, "leaky", False, 4096),
}
# fused Residual(DilatedUnit): name: (C, d, t per clip)
UNITS = {"unit_64": (64, 9, 4096), "unit_128": (128, 3, 1024), "unit_256": (256, 3, 256),
         "unit_512": (512, 3, 128)}
PREC = 0


STAMPS = os.environ.get("RAVE_AMD_DIAG_LIB") == "1"


def stamp_report(s_, sums=False):
    """sums: conv stamps -- slots 0-4 are clock stamps, 5 and 6 wave 0's summed
    cycles in the K loop's weight waits and chunk-end window waits + barriers."""
    s_ = s_[s_[:, 7] != 0].astype(np.float64)
    if not len(s_):
        return
    rt = (s_[:, 7] - s_[:, 7].min()) * 10.0 / 1e3   # us (100 MHz)
    q = lambda v: f"{np.median(v):7.0f} [{np.percentile(v, 10):6.0f},{np.percentile(v, 90):6.0f}]"
    last = max(k for k in range(5 if sums else 7) if (s_[:, k] != 0).all())
    if sums:
        print(f"   K loop of wave 0, cycles: weight waits {q(s_[:, 5])}  chunk-end waits+barrier {q(s_[:, 6])}",
              flush=True)
    segs = "  ".join(f"s{k}-{k + 1} {q(s_[:, k + 1] - s_[:, k])}" for k in range(last))
    print(f"   WGs={len(s_)}  cycles median [p10,p90]: {segs}  total {q(s_[:, last] - s_[:, 0])}; "
          f"WG start spread {rt.max():.1f} us", flush=True)


def run_unit(name, B, iters, dev):
    C, d, T = UNITS[name]
    name0 = name
    rng = np.random.default_rng(0)
    w1 = (rng.standard_normal((C, C, 3)) / np.sqrt(3 * C)).astype(np.float32)
    w2 = (rng.standard_normal((C, C, 1)) / np.sqrt(C)).astype(np.float32)
    packed = torch.from_numpy(N.pack_unit_weight(w1, w2, C, precision=PREC)).to(dev)
    x = torch.randn(B, C, T, device=dev)
    y = torch.empty_like(x)
    b1, b2 = torch.randn(C, device=dev), torch.randn(C, device=dev)
    a = N.UnitArgs(channels=C, batch=B, t_len=T, dilation=d, pad_left=d, act=N.ACT["leaky"],
                   leaky_slope=0.2, precision=PREC, x=x.data_ptr(), x_sb=C * T, x_sc=T, y=y.data_ptr(),
                   y_sb=C * T, y_sc=T, weight=packed.data_ptr(), bias1=b1.data_ptr(), bias2=b2.data_ptr())
    ws = None
    nws = N.lib.rave_unit_workspace(C_.byref(a))
    if nws > 0 and os.environ.get("LB_UNIT_COOP", "1") != "0":   # cooperative form (C 256 / 512)
        ws = torch.zeros(nws, device=dev)
        a.workspace = ws.data_ptr()
        name = name + "_coop"
    st = C_.c_void_p(torch.cuda.current_stream().cuda_stream)
    stamps = None
    if STAMPS and PREC in (N.PREC_SPLIT16, N.PREC_F32_RING, N.PREC_BF16X3):
        stamps = torch.zeros(8 * 200000, dtype=torch.int64, device=dev)
        N.check(N.lib.rave_diag_unit_stamps(C_.c_void_p(stamps.data_ptr())))
    for _ in range(3):
        N.check(N.lib.rave_residual_unit(C_.byref(a), st))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        N.check(N.lib.rave_residual_unit(C_.byref(a), st))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    fl = 2.0 * B * T * C * C * 4
    mb = 3 * B * C * T * 4 / 1e6
    print(f"{name:12s} B={B}  {ms * 1e3:8.2f} us  {fl / ms / 1e9:7.2f} TFLOP/s  "
          f"{mb / ms / 1e3:6.2f} TB/s (x, y, residual)", flush=True)
    if stamps is not None:
        stamps.zero_()
        N.check(N.lib.rave_residual_unit(C_.byref(a), st))
        torch.cuda.synchronize()
        stamp_report(stamps.view(-1, 8).cpu().numpy())
        N.check(N.lib.rave_diag_unit_stamps(C_.c_void_p(0)))
    return ms


def cfg_str(c):
    if c == 0:
        return "heuristic"
    v = c - 1
    return f"tile{v & 15} S{((v >> 4) & 31) + 1}{' sep' if (v >> 9) & 1 else ''}"


def run(name, B, iters, dev, config=0):
    if name in UNITS:
        return run_unit(name, B, iters, dev)
    ci, co, k, s, d, tr, act, has_res, T = LAYERS[name]
    rng = np.random.default_rng(0)
    w = rng.uniform(-0.05, 0.05, (ci, co, k) if tr else (co, ci, k)).astype(np.float32)
    packed = torch.from_numpy(N.pack_conv_weight(w, ci, co, k, s, d, tr, precision=PREC)).to(dev)
    x = torch.randn(B, ci, T, device=dev)
    if tr:
        t_out, pl, pr = T * s, 0, 0
    else:
        p = (k - 1) * d + 1
        pl, pr = (p - 1) // 2, p // 2
        t_out = (T + pl + pr - p) // s + 1
    y = torch.empty(B, co, t_out, device=dev)
    res = torch.randn(B, co, t_out, device=dev) if has_res else None
    bias = torch.randn(co, device=dev)
    a = N.ConvArgs(c_in=ci, c_out=co, kernel=k, stride=s, dilation=d, pad_left=pl, pad_right=pr,
                   transposed=tr, out_shift=s // 2 if tr else 0, act=N.ACT[act], leaky_slope=0.2,
                   batch=B, t_in=T, t_out=t_out, precision=PREC, x=x.data_ptr(), x_sb=ci * T, x_sc=T,
                   y=y.data_ptr(), y_sb=co * t_out, y_sc=t_out,
                   residual=res.data_ptr() if res is not None else None, r_sb=co * t_out, r_sc=t_out,
                   weight=packed.data_ptr(), bias=bias.data_ptr(),
                   config=config if isinstance(config, int) else 0)
    if config == "all":
        a.config = 0
        res_ = {c: None for c in [0] + N.conv_configs(a)}
        for c in res_:
            res_[c] = run(name, B, iters, dev, c)
        best = min(res_, key=res_.get)
        print(f"  -> best {cfg_str(best)} {res_[best] * 1e3:.2f} us", flush=True)
        return res_[best]
    stamps = None
    if STAMPS:
        stamps = torch.zeros(8 * 200000, dtype=torch.int64, device=dev)
        a.stamps = stamps.data_ptr()
    nws = N.lib.rave_conv1d_workspace(C.byref(a))
    ws = torch.zeros(max(nws, 1), device=dev)
    if nws > 0:
        a.partial = ws.data_ptr()
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        N.check(N.lib.rave_conv1d(C.byref(a), st))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        N.check(N.lib.rave_conv1d(C.byref(a), st))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    taps = 2 if tr else k
    fl = 2.0 * B * co * t_out * ci * taps
    print(f"{name:12s} B={B} {cfg_str(config):16s} ws={nws:>9d}  {ms * 1e3:8.2f} us  "
          f"{fl / ms / 1e9:7.2f} TFLOP/s", flush=True)
    if stamps is not None:
        stamps.zero_()
        N.check(N.lib.rave_conv1d(C.byref(a), st))
        torch.cuda.synchronize()
        stamp_report(stamps.view(-1, 8).cpu().numpy(), sums=True)
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default=",".join(list(LAYERS) + list(UNITS)))
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--precision", default="split16", choices=["f32", "split16", "f32_ring", "bf16x3"])
    ap.add_argument("--config", default="0", help="launch config value, or 'all' (every listed one)")
    a = ap.parse_args()
    global PREC
    PREC = N.PRECISION[a.precision]
    dev = torch.device("cuda")
    for name in a.layers.split(","):
        run(name, a.batch, a.iters, dev, a.config if a.config == "all" else int(a.config))


if __name__ == "__main__":
    main()
