"""Per-launch byte model of the conv_split16 family against its PMC counters.

For every conv the bench step runs as a standalone split-f16 conv launch
(units the autotuner left unfused, strided / transposed convs, the edge convs),
two models of the bytes one launch moves between the XCD L2s and memory:

* algorithmic: weights W + input X + output Y (+ residual), each once;
* XCD-replicated weights: 8 W + X + Y -- the launch runs batch-major per XCD
  (csrc/common.h xcd_major), so each of the 8 XCDs reads its own batch items'
  activations once but every weight row its tiles need, i.e. all of W.

Compared with the FETCH_SIZE x2 + WRITE_SIZE counter average of
profiles/<tag>/traffic.json (which counts Infinity-Cache hits as well as HBM).
Usage: python tools/traffic_model.py profiles/r02_s6
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rave_amd.config import v2
from rave_amd.graph import build_graph


def main(prof: str) -> None:
    tun = json.load(open(os.path.join(prof, "tuning.json")))
    fuse = {r[0].split("|")[1]: r[1] for r in tun if r[0].startswith("fuse|")}
    traffic = json.load(open(os.path.join(prof, "traffic.json")))["families"]["conv_split16"]
    g = build_graph(v2())
    B, rows = 16, []
    for part, nodes, t in (("enc", g.encoder, 4096), ("dec", g.decoder, 64)):
        for n in nodes:
            to = n.out_len(t)
            if ".aligned." in n.name:
                head = n.name[: n.name.rfind(".net.")] + ".net.1"
                # an unfused unit runs its two convs as conv launches (a stacked
                # or fused unit runs none)
                standalone = fuse.get(head, 1) == 0
            else:
                standalone = True
            if standalone:
                w = n.c_in * n.c_out * n.kernel * 4
                x = B * n.c_in * t * 4
                y = B * n.c_out * to * 4 * (2 if n.residual else 1)
                rows.append((n.name, w, x, y))
            t = to
    k = len(rows)
    alg = sum(w + x + y for _, w, x, y in rows) / k
    rep = sum(8 * w + x + y for _, w, x, y in rows) / k
    print(json.dumps({"launches": k, "algorithmic_MB": round(alg / 1e6, 2),
                      "xcd_replicated_weights_MB": round(rep / 1e6, 2),
                      "counter_MB": round(traffic["bytes_per_launch"] / 1e6, 2),
                      "layers": [{"name": r[0], "W_MB": round(r[1] / 1e6, 2), "X_MB": round(r[2] / 1e6, 2),
                                  "Y_MB": round(r[3] / 1e6, 2)} for r in rows]}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/r02_s6")
