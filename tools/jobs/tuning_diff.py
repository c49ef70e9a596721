"""Per-key time of two tuning files (GPU job logs): the conv keys whose choice
changed, old -> new config and time, and the sum over the changed keys."""
import json
import sys

old = {k: (v, t) for k, v, t in json.load(open(sys.argv[1]))}
new = {k: (v, t) for k, v, t in json.load(open(sys.argv[2]))}
prefix = sys.argv[3] if len(sys.argv) > 3 else "conv|"


def desc(v):
    c = v % 65536
    if c == 0:
        return f"p{v // 65536}:heur"
    c -= 1
    return f"p{v // 65536}:t{c & 15}S{((c >> 4) & 31) + 1}{'s' if (c >> 9) & 1 else ''}pm{1 << ((c >> 10) & 3)}"


d_old = d_new = 0.0
for k in sorted(new):
    if not k.startswith(prefix) or k not in old:
        continue
    (vo, to), (vn, tn) = old[k], new[k]
    if vo != vn:
        d_old += to
        d_new += tn
        print(f"{k:60s} {desc(vo):18s} {to * 1e3:7.2f} -> {desc(vn):18s} {tn * 1e3:7.2f} us")
print(f"changed keys: {d_old * 1e3:.1f} -> {d_new * 1e3:.1f} us")
