"""MFMA utilisation per kernel family from one rocprofv3 --pmc pass with
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (tools/profile_round.sh).

* SQ_VALU_MFMA_BUSY_CYCLES: MFMA-pipe busy cycles summed over every SIMD
  (MI355X_MICROARCH.md: 32 per 32x32x16 f16/bf16 MFMA);
* GRBM_GUI_ACTIVE: GPU-busy cycles of the dispatch summed over the 8 XCDs.

utilisation = MFMA busy / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs): the fraction of
the chip's MFMA issue slots the family's launches kept busy, padding included.
``expected_busy`` is what the family's algorithmic FLOP need at 1024 FLOP per
SIMD-cycle (x3 for split-f16: three f16 MFMAs per fp32 MAC); busy above it is
MFMA work on padded rows/columns.
Usage: python tools/mfma_util.py <counter_collection.csv> [bench.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rocprof_summary import FAMILIES, classify, set_precision  # noqa: E402

SIMDS = 1024          # 256 CUs x 4 SIMDs
FLOP_PER_SIMD_CYCLE = 1024.0   # dense f16 MFMA: 2516.6 TFLOP/s / (1024 SIMDs x 2.4 GHz)


def main(path, bench=None):
    if bench:      # exact-fp32 runs: the edges and the split-K reduce belong to fp32 families
        set_precision(json.load(open(bench)).get("precision", "auto"))
    busy, active, launches = defaultdict(float), defaultdict(float), defaultdict(set)
    with open(path, newline="") as fh:
        for r in csv.DictReader(fh):
            fam, main = classify(r["Kernel_Name"])
            if fam not in FAMILIES:
                continue
            v = float(r["Counter_Value"])
            if r["Counter_Name"] == "SQ_VALU_MFMA_BUSY_CYCLES":
                busy[fam] += v
            elif r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                active[fam] += v
            if main:
                launches[fam].add(r["Dispatch_Id"])
    flop = {}
    if bench:
        d = json.load(open(bench))
        fams = dict(d["roofline"]["families"])
        for side in ("f32_exact", "split16_auto"):
            fams.update(((d.get(side) or {}).get("roofline") or {}).get("families") or {})
        for f, v in fams.items():
            flop[f] = v.get("flop_per_launch_avg")
    out = {}
    for f in sorted(busy, key=lambda q: -busy[q]):
        n = len(launches[f]) or 1
        cyc = active[f] / 8.0
        rec = {"launches": n, "mfma_busy_cycles_per_launch": round(busy[f] / n),
               "gpu_cycles_per_launch": round(cyc / n),
               "mfma_utilisation": round(busy[f] / (cyc * SIMDS), 4) if cyc else None}
        if flop.get(f):
            # f16 MFMA passes per fp32 MAC: split16 3, bf16x3 6 (bf16 rate = f16 rate);
            # the fp32 MFMA runs at 1/16 of the f16 rate
            mult = 3.0 if f.endswith("split16") else 6.0 if f.endswith("bf16x3") else 16.0
            if f == "tail_bf16x3" and d.get("tail_synthesis") == "f32":
                # round 5's tail: its conv (14336 MACs per frame) in bf16x3, its synthesis
                # (8448) in fp32 (since round 6 both in bf16x3: mult 6)
                mult = (14336 * 6.0 + 8448 * 16.0) / (14336 + 8448)
            if f == "head_bf16x3":
                # its analysis (6 bands x 513 taps: 3078 MACs per frame) in bf16x3, its
                # conv (64 x 6 x 7: 2688) in exact fp32
                mult = (3078 * 6.0 + 2688 * 16.0) / (3078 + 2688)
            rec["expected_busy_per_launch"] = round(flop[f] * mult / FLOP_PER_SIMD_CYCLE)
            rec["busy_over_expected"] = round(busy[f] / n / rec["expected_busy_per_launch"], 3)
        out[f] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
