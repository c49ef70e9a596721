#!/usr/bin/env python3
"""Per-kernel anatomy of one C3 streaming block (BASELINE configs[2]: v2 causal,
B = 1, 2048-sample blocks), for rocprofv3 --kernel-trace.

    rocprofv3 --kernel-trace --output-format csv -d D -o run -- python3 tools/c3_trace.py run
    python3 tools/c3_trace.py summarize D/.../run_kernel_trace.csv > c3_ops.json

``run`` builds the stream plans (autotuning launches happen here), then fires a
marker kernel (torch cumsum of a 7-element tensor: a scan) and streams BLOCKS eager
encode+decode blocks; ``summarize`` keeps the dispatches after the last marker
and reports, per kernel name, launches per block and the mean duration, plus
the first block's launch sequence with start-to-start gaps.
"""
import csv
import json
import os
import sys
from collections import defaultdict

BLOCKS = 40


def run():
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    dev = torch.device("cuda:0")
    cfg = rcfg.causal()
    prec = os.environ.get("C3_PRECISION", "auto")
    m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=prec)
    s = StreamingRAVE(m, batch=1, block=2048, graph=False)
    x = (0.2 * torch.randn(BLOCKS + 4, 1, 1, 2048, generator=torch.Generator().manual_seed(0))).to(dev)
    for i in range(4):
        s.forward(x[i])
    torch.cuda.synchronize()
    torch.arange(7, device=dev).cumsum(0)     # marker (a scan kernel: no rave kernel is one)
    torch.cuda.synchronize()
    for i in range(BLOCKS):
        s.forward(x[4 + i])
        torch.cuda.synchronize()
    print(json.dumps({"blocks": BLOCKS, "precision": prec}))


def summarize(path):
    with open(path, newline="") as fh:
        rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Start_Timestamp"]))
    def is_marker(r):
        k = r["Kernel_Name"].lower()
        return "rave" not in k and ("scan" in k or "cumsum" in k)
    last = max(i for i, r in enumerate(rows) if is_marker(r))
    rows = rows[last + 1:]
    name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "")[:90]
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in rows:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        tot[name(r)] += d
        cnt[name(r)] += 1
    per_block = len(rows) / BLOCKS
    ker = sorted(tot, key=lambda k: -tot[k])
    out = {"launches_per_block": per_block,
           "busy_us_per_block": sum(tot.values()) / BLOCKS / 1e3,
           "span_us_per_block": (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / BLOCKS / 1e3,
           "kernels": [{"kernel": k, "per_block": cnt[k] / BLOCKS, "avg_us": tot[k] / cnt[k] / 1e3,
                        "us_per_block": tot[k] / BLOCKS / 1e3} for k in ker]}
    n = int(round(per_block))
    seq, t_prev = [], None
    for r in rows[:n]:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        seq.append({"kernel": name(r), "us": (en - st) / 1e3, "gap_us": (st - t_prev) / 1e3 if t_prev else 0.0})
        t_prev = en
    out["first_block"] = seq
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        summarize(sys.argv[2])
