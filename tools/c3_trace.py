#!/usr/bin/env python3
"""Where a C3 streaming block's time goes (BASELINE configs[2]: v2 causal,
2048-sample blocks, B = 1), from a rocprofv3 kernel trace.

    run:      rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- \
                  python3 tools/c3_trace.py run --precision f32_bf3
    analyse:  python3 tools/c3_trace.py analyse OUT/.../run_kernel_trace.csv

``run`` builds the causal model with the committed launch choices
(profiles/tuning/c3_<precision>.json, as bench.py's configs leg), replays
``--blocks`` encode+decode blocks after 8 warm-up blocks with a synchronize
around each (the latency measurement), and prints the host latencies as JSON.
``analyse`` splits the trace into blocks at the host gaps and reports, per
block: the span (first kernel start to last kernel end), the kernels' busy time
and the gaps between them, plus each kernel's mean duration -- the part of the
block latency the kernels themselves take against what the launches and the
host add."""
import argparse
import csv
import json
import os
import sys
import time
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run(a):
    import numpy as np
    import torch
    from bench import _pinned
    from rave_amd import config as rcfg
    from rave_amd.model import RAVE
    from rave_amd.streaming import StreamingRAVE
    from rave_amd.weights import init_params, init_speaker
    dev = torch.device("cuda:0")
    cfg = rcfg.causal()
    tun, src = (None, "autotuned at plan build") if a.retune else _pinned("c3", a.precision)
    if a.tuning:
        with open(a.tuning) as fh:
            tun, src = json.load(fh), a.tuning
    m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=a.precision, tuning=tun)
    blk, warm, nb = 2048, 8, a.blocks
    x = (0.2 * torch.randn(warm + nb, 1, 1, blk, generator=torch.Generator().manual_seed(0))).to(dev)
    s = StreamingRAVE(m, batch=1, block=blk, graph=True)
    s.reset()
    lat = []
    for i in range(warm + nb):
        torch.cuda.synchronize()
        if a.sleep_ms > 0:
            time.sleep(a.sleep_ms / 1e3)        # a wider gap between blocks in the trace
        t0 = time.perf_counter()
        s.forward(x[i])
        torch.cuda.synchronize()
        if i >= warm:
            lat.append((time.perf_counter() - t0) * 1e3)
    lat = np.array(lat)
    if a.save:
        with open(a.save, "w") as fh:
            json.dump(m.tuning(), fh, indent=0)
    print(json.dumps({"precision": a.precision, "tuning": src, "blocks": nb,
                      "launches": {"encode": s.launches("encode"), "decode": s.launches("decode")},
                      "latency_ms_median": round(float(np.median(lat)), 4),
                      "latency_ms_p99": round(float(np.percentile(lat, 99)), 4)}))


def analyse(a):
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    blocks, cur = [], []
    for r in rows:
        if cur and r[0] - cur[-1][1] > a.gap_us * 1000:
            blocks.append(cur)
            cur = []
        cur.append(r)
    if cur:
        blocks.append(cur)
    # the timed blocks: the last ones of the modal kernel count (warm-up and plan
    # building launch other kernels)
    counts = defaultdict(int)
    for b in blocks:
        counts[len(b)] += 1
    n_mode = max(counts, key=lambda k: (counts[k], k))
    timed = [b for b in blocks if len(b) == n_mode][-a.blocks:]
    spans = sorted((b[-1][1] - b[0][0]) / 1e3 for b in timed)
    busy = sorted(sum(e - s for s, e, _ in b) / 1e3 for b in timed)
    per = defaultdict(list)
    for b in timed:
        for i, (s, e, n) in enumerate(b):
            per[(i, n)].append((e - s) / 1e3)
    mid = len(timed) // 2
    out = {"blocks": len(timed), "kernels_per_block": n_mode,
           "span_us_median": round(spans[mid], 1), "busy_us_median": round(busy[mid], 1),
           "gaps_us_median": round(spans[mid] - busy[mid], 1),
           "kernels": [{"i": i, "name": n.split("(")[0][:90], "us": round(sorted(v)[len(v) // 2], 2)}
                       for (i, n), v in sorted(per.items())]}
    print(json.dumps(out, indent=1))


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--precision", default="f32_bf3")
    r.add_argument("--blocks", type=int, default=32)
    r.add_argument("--retune", action="store_true", help="time every launch choice instead of the pins")
    r.add_argument("--save", help="write the plan's launch choices (RAVE.tuning()) here")
    r.add_argument("--tuning", help="launch choices to replay instead of the committed pins")
    r.add_argument("--sleep-ms", type=float, default=0.0,
                   help="host sleep before each block (the bench leg has none: clocks stay up)")
    an = sub.add_parser("analyse")
    an.add_argument("trace")
    an.add_argument("--blocks", type=int, default=32)
    an.add_argument("--gap-us", type=float, default=15.0)
    a = ap.parse_args()
    run(a) if a.cmd == "run" else analyse(a)


if __name__ == "__main__":
    main()
