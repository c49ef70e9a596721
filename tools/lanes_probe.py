"""Probe: one bench step (16 x 65536 v2 encode+decode, f32_bf3) run as L
micro-batches of 16/L clips on L HIP streams (one engine instance each, joined
at the end of the step) against the one-stream step.  Prints ms/step per L,
interleaved over rounds.  Tuning: the pinned B=16 file for L=1; the B=16/L
plans are timed at plan build once (first lane) and replayed by the others."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402
from rave_amd import config as rcfg  # noqa: E402
from rave_amd.model import RAVE  # noqa: E402
from rave_amd.weights import init_params, init_speaker  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", default="1,2,4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--precision", default="f32_bf3")
    ap.add_argument("--tuning-out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = rcfg.v2()
    params, spk = init_params(cfg, seed=0), init_speaker(cfg, seed=0)
    B, T = 16, 65536
    x = torch.from_numpy(bench.synth_batch(B, T, 0)).to(dev)
    pinned = bench.tuning_path(cfg.name, B, T, a.precision)
    setups = {}
    tunings = {}
    for L in [int(v) for v in a.lanes.split(",")]:
        tun = json.load(open(pinned)) if (L == 1 and os.path.exists(pinned)) else None
        t0 = time.perf_counter()
        m0 = RAVE(cfg, params, spk, device=dev, precision=a.precision, tuning=tun)
        xs = list(torch.chunk(x, L, dim=0))
        m0.decode(m0.encode(xs[0]))          # builds (and times) the B/L plans
        torch.cuda.synchronize()
        models = [m0] + [RAVE(cfg, params, spk, device=dev, precision=a.precision, tuning=m0.tuning())
                         for _ in range(L - 1)]
        streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(L - 1)]
        tunings[L] = m0.tuning()
        print(f"L={L}: plans built in {time.perf_counter() - t0:.1f} s, {len(tunings[L])} tuning entries",
              flush=True)
        setups[L] = (models, streams, xs)

    def step(L):
        models, streams, xs = setups[L]
        main = streams[0]
        ev = torch.cuda.Event()
        ev.record(main)
        outs = []
        for m, s, xi in zip(models, streams, xs):
            s.wait_event(ev)
            with torch.cuda.stream(s):
                outs.append(m.decode(m.encode(xi)))
        for s in streams[1:]:
            main.wait_stream(s)
        return outs

    ref = torch.cat(step(1), 0) if 1 in setups else None
    for L in setups:
        y = torch.cat(step(L), 0)
        torch.cuda.synchronize()
        if ref is not None:
            print(f"L={L}: max |y - y(L=1)| = {float((y - ref).abs().max()):.3e}", flush=True)
    for r in range(a.rounds):
        for L in setups:
            for _ in range(3):
                step(L)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step(L)
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / a.steps
            print(f"round {r} L={L}: {el * 1e3:.4f} ms/step  {B * T / el / 1e9:.3f} G samples/s", flush=True)
        for m in setups[max(setups)][0]:
            m.check()
    if a.tuning_out:
        json.dump({str(k): v for k, v in tunings.items()}, open(a.tuning_out, "w"))


if __name__ == "__main__":
    main()
