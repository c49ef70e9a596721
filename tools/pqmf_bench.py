#!/usr/bin/env python3
"""Time the PQMF synthesis kernel at config-2 size (16 x 4096 frames, AM epilogue);
with RAVE_AMD_DIAG_LIB=1 also print per-workgroup phase stamps."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rave_amd import _native as N  # noqa: E402
from tools.layer_bench import stamp_report  # noqa: E402

dev = torch.device("cuda")
B, F = 16, 4096
x = torch.randn(B, 32, F, device=dev)
y = torch.empty(B, 1, F * 16, device=dev)
hki = torch.randn(16, 16, 33, device=dev)
a = N.SynthesisArgs(n_band=16, taps=33, batch=B, t_in=F, pad_left=16, mode=1, frame0=0, x_len=0,
                    x=x.data_ptr(), x_sb=32 * F, x_sc=F, y=y.data_ptr(), y_sb=F * 16, hki=hki.data_ptr())
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(3):
    N.check(N.lib.rave_pqmf_synthesis(C.byref(a), st))
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    N.lib.rave_pqmf_synthesis(C.byref(a), st)
e1.record()
torch.cuda.synchronize()
print(f"synthesis {e0.elapsed_time(e1) / 20 * 1e3:.2f} us")
if os.environ.get("RAVE_AMD_DIAG_LIB") == "1":
    s = torch.zeros(8 * 4096, dtype=torch.int64, device=dev)
    N.check(N.lib.rave_diag_pqmf_stamps(C.c_void_p(s.data_ptr())))
    N.check(N.lib.rave_pqmf_synthesis(C.byref(a), st))
    torch.cuda.synchronize()
    stamp_report(s.view(-1, 8).cpu().numpy())
