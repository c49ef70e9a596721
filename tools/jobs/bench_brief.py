"""One-screen summary of a bench.py JSON line (GPU job logs)."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d.get("roofline") or {}
fams = r.get("families") or {}
if "--short" in sys.argv:
    print(d["ms_per_step"], "ms/step;", " ".join(f"{k}={v['launches']}x{v['avg_launch_ms'] * 1e3:.1f}us"
                                                   for k, v in fams.items()))
    sys.exit(0)
print("headline", d["precision"], d["ms_per_step"], "ms/step", d["value"], "samples/s; roofline", r.get("kernel"),
      r.get("frac"))
print("launches", d["gemm_launches_by_family"], "tuning", d["tuning"])
for side in ("f32_exact", "split16_auto", "pipelined"):
    v = d.get(side) or {}
    print(side, v.get("ms_per_step"), {k: v[k] for k in v if k.endswith("max_abs")})
print("cpu", d.get("cpu_baseline"))
for k, v in fams.items():
    print(f"  {k:14s} {v['launches']:3d} x {v['avg_launch_ms'] * 1e3:7.2f} us  frac {v['frac']:.3f}  "
          f"{v['achieved']} {v['unit']}")
