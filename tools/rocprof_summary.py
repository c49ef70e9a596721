#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output of ``bench.py`` for the conv roofline.

    python tools/rocprof_summary.py --trace KT.csv [--fetch FETCH.csv] [--write WRITE.csv] \
        [--bench BENCH.json] [--out SUMMARY.json]

* ``--trace``: a ``*_kernel_trace.csv`` (rocprofv3 --kernel-trace).  One conv
  op of a plan is the main ``conv1d_mfma_kernel`` launch plus, when split-K is
  used, its ``conv1d_splitk_reduce_kernel``; the per-op duration is
  (sum of both kernels) / (number of main launches) -- the same quantity
  bench.py's HIP events time per conv op.
* ``--fetch`` / ``--write``: ``*_counter_collection.csv`` of two separate
  ``--pmc FETCH_SIZE`` / ``--pmc WRITE_SIZE`` passes (the counters do not fit
  one pass on gfx950).  FETCH_SIZE is doubled (gfx950 tallies 128-B
  requests at 64 B, MI355X_MICROARCH.md "HBM"); both are in KB.  Traffic per
  conv op = (2*FETCH + WRITE) over the conv kernels / main launches.
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict

MAIN = "conv1d_mfma_kernel"
REDUCE = "conv1d_splitk_reduce_kernel"


def _rows(path):
    with open(path, newline="") as fh:
        return list(csv.DictReader(fh))


def kernel_family(name: str) -> str:
    for fam in (MAIN, REDUCE, "pqmf_analysis_kernel", "pqmf_synthesis_kernel", "fill_channels_kernel",
                "rvq_encode_kernel", "rvq_decode_kernel", "noise_synth_kernel", "adain_kernel",
                "copy_kernel", "shift_history_kernel"):
        if fam in name:
            return fam
    return name.split("(")[0][:60]


def trace_summary(path):
    fam_ns = defaultdict(float)
    fam_n = defaultdict(int)
    for r in _rows(path):
        ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        f = kernel_family(r["Kernel_Name"])
        fam_ns[f] += ns
        fam_n[f] += 1
    n_main = fam_n.get(MAIN, 0)
    conv_ns = fam_ns.get(MAIN, 0.0) + fam_ns.get(REDUCE, 0.0)
    return {
        "families": {f: {"calls": fam_n[f], "total_ms": round(fam_ns[f] / 1e6, 4),
                         "avg_us": round(fam_ns[f] / fam_n[f] / 1e3, 3)}
                     for f in sorted(fam_ns, key=lambda k: -fam_ns[k])},
        "conv_ops": n_main,
        "conv_avg_op_ms": conv_ns / n_main / 1e6 if n_main else None,
        "conv_main_avg_ms": fam_ns.get(MAIN, 0.0) / n_main / 1e6 if n_main else None,
    }


def counter_total(path, counter):
    """Sum of a counter over conv kernels (main + reduce) and the main-launch count."""
    tot = 0.0
    seen = set()
    for r in _rows(path):
        if r.get("Counter_Name") != counter:
            continue
        f = kernel_family(r["Kernel_Name"])
        if f in (MAIN, REDUCE):
            tot += float(r["Counter_Value"])
            if f == MAIN:
                seen.add(r["Dispatch_Id"])
    return tot, len(seen)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--bench", help="bench.py JSON line to compare the event average with")
    ap.add_argument("--out")
    ap.add_argument("--traffic-out", help="write bench.py's profiles/conv_traffic.json")
    ap.add_argument("--workload", default="v2,16,65536", help="config,batch,samples of the passes")
    a = ap.parse_args()
    s = trace_summary(a.trace)
    if a.fetch and a.write:
        fkb, nf = counter_total(a.fetch, "FETCH_SIZE")
        wkb, nw = counter_total(a.write, "WRITE_SIZE")
        s["traffic"] = {
            "fetch_bytes_per_op": 2.0 * fkb * 1024 / nf,
            "write_bytes_per_op": wkb * 1024 / nw,
            "bytes_per_op": 2.0 * fkb * 1024 / nf + wkb * 1024 / nw,
            "ops_fetch_pass": nf, "ops_write_pass": nw,
            "note": "FETCH_SIZE x2 (gfx950 correction); KB -> bytes; conv main + split-K reduce",
        }
    if a.bench:
        with open(a.bench) as fh:
            b = json.loads(fh.read().strip().splitlines()[-1])
        ev = b["roofline"]["avg_launch_ms"]
        s["bench_event_avg_op_ms"] = ev
        s["rocprof_vs_event"] = s["conv_avg_op_ms"] / ev if ev else None
    if a.traffic_out and "traffic" in s:
        cfg, b, t = a.workload.split(",")
        with open(a.traffic_out, "w") as fh:
            json.dump({"workload": [cfg, int(b), int(t)], "bytes_per_op": round(s["traffic"]["bytes_per_op"]),
                       "fetch_bytes_per_op": round(s["traffic"]["fetch_bytes_per_op"]),
                       "write_bytes_per_op": round(s["traffic"]["write_bytes_per_op"]),
                       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of bench.py "
                                 "(tools/profile_round.sh); FETCH_SIZE x2 gfx950 correction"}, fh, indent=1)
    txt = json.dumps(s, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
