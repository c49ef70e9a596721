#!/usr/bin/env python3
"""Per-op HIP-event times of one model plan (the engine's rave_model_profile),
sorted by time: where a config's step goes.

    python tools/plan_ops.py --config discrete --plan encode_codes --batch 8 --samples 65536
    python tools/plan_ops.py --config v2 --plan decode --batch 16 --precision f32_tuned \
        --tuning-in profiles/tuning/v2_16x65536_f32_tuned.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rave_amd import config as rcfg  # noqa: E402
from rave_amd.model import DECODE, DECODE_CODES, ENCODE, ENCODE_CODES, RAVE  # noqa: E402
from rave_amd.weights import init_params, init_speaker  # noqa: E402

PLANS = {"encode": ENCODE, "decode": DECODE, "encode_codes": ENCODE_CODES, "decode_codes": DECODE_CODES}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="discrete")
    ap.add_argument("--plan", default="encode_codes", choices=list(PLANS))
    ap.add_argument("--precision", default="auto")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--samples", type=int, default=65536)
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--tuning-in", help="JSON of RAVE.tuning() (e.g. profiles/tuning/*.json): the pinned launch choices")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = rcfg.get_config(a.config)
    tuning = None
    if a.tuning_in:
        with open(a.tuning_in) as fh:
            tuning = json.load(fh)
    m = RAVE(cfg, init_params(cfg, 0), init_speaker(cfg, 0), device=dev, precision=a.precision, tuning=tuning)
    B, T = a.batch, a.samples
    x = (0.2 * torch.randn(B, 1, T, generator=torch.Generator().manual_seed(0))).to(dev)
    which = PLANS[a.plan]
    if which in (ENCODE, ENCODE_CODES):
        run, t = ((lambda: m.encode(x)) if which == ENCODE else (lambda: m.encode_codes(x))), T
    else:
        z = m.encode(x) if which == DECODE else m.encode_codes(x)
        run, t = ((lambda: m.decode(z)) if which == DECODE else (lambda: m.decode_codes(z))), T // cfg.hop
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    ops = m.ops(which, B, t)
    m.profile(which, B, t, a.runs)
    for _ in range(a.runs):
        run()
    torch.cuda.synchronize()
    ms, n = m.op_times(which, B, t)
    m.profile(which, B, t, 0)
    rows = sorted(({"label": o["label"], "kind": o["kind"], "precision": o["precision"],
                    "us": round(float(v) / n * 1e3, 2)} for o, v in zip(ops, ms)), key=lambda r: -r["us"])
    print(json.dumps({"config": a.config, "plan": a.plan, "precision": a.precision, "batch": B, "samples": T,
                      "ops": len(ops), "sum_us": round(sum(r["us"] for r in rows), 1), "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
