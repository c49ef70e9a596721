#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output of ``bench.py`` for the roofline line.

    python tools/rocprof_summary.py --trace KT.csv [--fetch FETCH.csv] [--write WRITE.csv] \
        [--bench BENCH.json] [--out SUMMARY.json] [--traffic-out TRAFFIC.json]

* ``--trace``: a ``*_kernel_trace.csv`` (rocprofv3 --kernel-trace).  Kernels
  are grouped into the GEMM families bench.py reports (``FAMILIES``): one op
  of a family is its main kernel launch plus, for the convs, the split-K
  reduce launched after it when the op splits K; the per-op duration is
  (sum over the family's kernels) / (number of main launches) -- the same
  quantity bench.py's HIP events time per op.
* ``--fetch`` / ``--write``: ``*_counter_collection.csv`` of two separate
  ``--pmc FETCH_SIZE`` / ``--pmc WRITE_SIZE`` passes (the counters do not fit
  one pass on gfx950).  FETCH_SIZE is doubled (gfx950 tallies 128-B
  requests at 64 B, MI355X_MICROARCH.md "HBM"); both are in KB.  Traffic per
  op launch = (2*FETCH + WRITE) over the family's kernels / main launches.
"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict

# family -> (main kernels, helper kernels launched by the same op)
FAMILIES = {
    "conv_f32": (("conv1d_mfma_kernel", "conv1d_ring_f32_kernel"), ("conv1d_splitk_reduce_kernel",)),
    "conv_split16": (("conv1d_split_kernel",), ("split_reduce_kernel",)),
    "unit_f32": (("residual_unit_kernel", "unit_ring_f32_kernel"), ()),
    "unit_split16": (("unit_split_kernel",), ()),
    "conv_bf16x3": (("conv1d_bf3_kernel",), ()),
    "unit_bf16x3": (("unit_bf3_kernel",), ()),
    "stack_split16": (("stack_split_kernel",), ()),
    "stack_bf16x3": (("stack_bf3_kernel",), ()),
    "pqmf_analysis_f32": (("pqmf_analysis_kernel",), ()),
    "pqmf_synthesis_f32": (("pqmf_synthesis_kernel",), ()),
    "pqmf_analysis_split16": (("pqmf_analysis_split_kernel",), ()),
    "pqmf_synthesis_split16": (("pqmf_synthesis_split_kernel",), ()),
    "head_split16": (("encoder_head_kernel",), ()),
    "tail_split16": (("decoder_tail_kernel",), ()),
    "head_f32": ((), ()),
    "tail_f32": ((), ()),
    "tail_bf16x3": ((), ()),
    "head_bf16x3": ((), ()),
}
_KERNEL_FAMILY = {}
for _fam, (_mains, _helpers) in FAMILIES.items():
    for _m in _mains:
        _KERNEL_FAMILY[_m] = (_fam, True)
    for _h in _helpers:
        _KERNEL_FAMILY[_h] = (_fam, False)


def set_precision(precision: str) -> None:
    """Exact-fp32 runs: the split kernels' separate K-split reduce belongs to
    the fp32 ring convs (conv1d_ring_f32_kernel), not to a split16 family."""
    if precision == "f32_bf3":
        # (the split kernels' reduce: counted with the bf16x3 convs, which take most split-K launches)
        _KERNEL_FAMILY["split_reduce_kernel"] = ("conv_bf16x3", False)
        _KERNEL_FAMILY["encoder_head_kernel"] = ("head_f32", True)
        _KERNEL_FAMILY["decoder_tail_kernel"] = ("tail_f32", True)
    if precision in ("f32", "f32_tuned"):
        _KERNEL_FAMILY["split_reduce_kernel"] = ("conv_f32", False)
        _KERNEL_FAMILY["encoder_head_kernel"] = ("head_f32", True)     # the edges' exact-fp32 form
        _KERNEL_FAMILY["decoder_tail_kernel"] = ("tail_f32", True)


_NAME = re.compile(r"(?:^|[\s:])([A-Za-z_][A-Za-z0-9_]*)\s*[<(]")


def _rows(path):
    with open(path, newline="") as fh:
        return list(csv.DictReader(fh))


def kernel_name(demangled: str) -> str:
    """Bare function name of a demangled kernel symbol
    ('void rave::conv1d_split_kernel<3, 64>(rave::ConvKArgs)' -> 'conv1d_split_kernel')."""
    m = _NAME.search(demangled)
    return m.group(1) if m else demangled.split("(")[0][:60]


_TAIL_AR = re.compile(r"decoder_tail_kernel<[^<>]*,\s*([012])>")
_HEAD_AR = re.compile(r"encoder_head_kernel<\s*([012])\s*>")


def classify(demangled: str):
    """(family or bare kernel name, is the family's main launch)."""
    k = kernel_name(demangled)
    if k == "decoder_tail_kernel":
        # round 5: the last template argument is the arithmetic (0 split16, 1 exact
        # fp32, 2 bf16x3 conv + exact-fp32 synthesis); older builds had a bool there
        m = _TAIL_AR.search(demangled)
        if m:
            return ({"0": "tail_split16", "1": "tail_f32", "2": "tail_bf16x3"}[m.group(1)], True)
    if k == "encoder_head_kernel":
        # round 6: the template argument is the arithmetic (0 split16, 1 exact fp32,
        # 2 bf16x3 analysis + exact-fp32 conv); older builds had a bool there
        m = _HEAD_AR.search(demangled)
        if m:
            return ({"0": "head_split16", "1": "head_f32", "2": "head_bf16x3"}[m.group(1)], True)
    return _KERNEL_FAMILY.get(k, (k, False))


def trace_summary(path):
    k_ns, k_n = defaultdict(float), defaultdict(int)
    fam_ns, fam_main = defaultdict(float), defaultdict(int)
    for r in _rows(path):
        ns = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        k = kernel_name(r["Kernel_Name"])
        k_ns[k] += ns
        k_n[k] += 1
        fam, main = classify(r["Kernel_Name"])
        if fam in FAMILIES:
            fam_ns[fam] += ns
            fam_main[fam] += int(main)
    return {
        "kernels": {k: {"calls": k_n[k], "total_ms": round(k_ns[k] / 1e6, 4),
                        "avg_us": round(k_ns[k] / k_n[k] / 1e3, 3)}
                    for k in sorted(k_ns, key=lambda q: -k_ns[q])},
        "families": {f: {"ops": fam_main[f], "total_ms": round(fam_ns[f] / 1e6, 4),
                         "avg_op_ms": fam_ns[f] / fam_main[f] / 1e6 if fam_main[f] else None}
                     for f in sorted(fam_ns, key=lambda q: -fam_ns[q])},
    }


def counter_by_family(path, counter):
    """Per family: sum of ``counter`` over its kernels and its main-launch count."""
    tot = defaultdict(float)
    seen = defaultdict(set)
    for r in _rows(path):
        if r.get("Counter_Name") != counter:
            continue
        fam, main = classify(r["Kernel_Name"])
        if fam in FAMILIES:
            tot[fam] += float(r["Counter_Value"])
            if main:
                seen[fam].add(r["Dispatch_Id"])
    return {f: (tot[f], len(seen[f])) for f in tot}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--bench", help="bench.py JSON line to compare the event averages with")
    ap.add_argument("--out")
    ap.add_argument("--traffic-out", help="write bench.py's profiles/traffic.json")
    ap.add_argument("--workload", default="v2,16,65536", help="config,batch,samples of the passes")
    ap.add_argument("--precision", default="auto", help="bench.py --precision of the passes")
    a = ap.parse_args()
    set_precision(a.precision)
    s = trace_summary(a.trace)
    if a.fetch and a.write:
        fe = counter_by_family(a.fetch, "FETCH_SIZE")
        wr = counter_by_family(a.write, "WRITE_SIZE")
        tr = {}
        for f in sorted(set(fe) & set(wr)):
            (fkb, nf), (wkb, nw) = fe[f], wr[f]
            if nf and nw:
                fb, wb = 2.0 * fkb * 1024 / nf, wkb * 1024 / nw
                tr[f] = {"bytes_per_launch": round(fb + wb), "fetch_bytes_per_launch": round(fb),
                         "write_bytes_per_launch": round(wb), "launches_fetch_pass": nf,
                         "launches_write_pass": nw}
        s["traffic"] = {"families": tr,
                        "note": "FETCH_SIZE x2 (gfx950 correction); KB -> bytes; main kernel + "
                                "its split-K reduce, per main launch"}
    if a.bench:
        with open(a.bench) as fh:
            b = json.loads(fh.read().strip().splitlines()[-1])
        cmp = {}
        for f, v in (b.get("roofline") or {}).get("families", {}).items():
            rp = s["families"].get(f, {}).get("avg_op_ms")
            ev = v.get("avg_launch_ms")
            cmp[f] = {"event_avg_op_ms": ev, "rocprof_avg_op_ms": rp,
                      "rocprof_over_event": rp / ev if rp and ev else None}
        s["rocprof_vs_event"] = cmp
    if a.traffic_out and "traffic" in s:
        cfg, bb, t = a.workload.split(",")
        with open(a.traffic_out, "w") as fh:
            json.dump({"workload": [cfg, int(bb), int(t)], "precision": a.precision,
                       "families": s["traffic"]["families"],
                       "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of bench.py "
                                 "(tools/profile_round.sh); FETCH_SIZE x2 gfx950 correction"}, fh, indent=1)
    txt = json.dumps(s, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
