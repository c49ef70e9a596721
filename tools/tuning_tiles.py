"""Print the split-conv tile / split-K choice of every autotuned conv in a
tuning file written by bench.py --tuning-out (config code = 1 + tile +
16 (S - 1) + 512 sep, csrc/conv_shared.h encode_config; precision in the high
16 bits)."""
import json
import sys

rows = json.load(open(sys.argv[1]))
rows = rows if isinstance(rows, list) else rows.get("entries", [])
for key, code, ms in rows:
    if not key.startswith("conv"):
        continue
    prec, cfg = divmod(code, 65536)
    if cfg == 0:
        desc = "default"
    else:
        c = cfg - 1
        desc = f"tile {c % 16} S {(c % 512) // 16 + 1} sep {c // 512}"
    print(f"{key:64s} prec {prec} {desc:24s} {ms * 1000:6.1f} us")
