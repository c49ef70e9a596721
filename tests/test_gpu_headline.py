"""The bench headline's own plan against the float64 oracle.

bench.py times ``--precision f32_bf3`` at BASELINE configs[1] (v2, 16 x 65536
per GPU) with its launch choices pinned by
``profiles/tuning/v2_16x65536_f32_bf3.json`` (cooperative bf16x3 units at
C = 256 / 512, bf16x3 convs, exact-fp32 path edges).  These tests build exactly
that plan -- the same weights (seed 0), the same synthetic clips
(bench.synth_batch) and the same pinned tuning, with no launch choice re-timed
-- and check it where the bench cannot: against the oracle
(oracle/rave_oracle.py, float64; rave/model.py:594-634), clip by clip, plus
batch independence and bitwise determinism at the full batch.

Tolerance: the north star's 1e-4 max-abs on model outputs."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

TOL = 1e-4
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, T = 16, 65536


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _tuning_file(precision):
    return os.path.join(REPO, "profiles", "tuning", f"v2_{B}x{T}_{precision}.json")


@pytest.fixture(scope="module")
def headline(dev):
    """The bench's f32_bf3 model on its pinned plan, its input and one output."""
    from bench import synth_batch
    from rave_amd import _native as N
    from rave_amd import config as rcfg
    from rave_amd.model import DECODE, ENCODE, RAVE
    from rave_amd.weights import init_params, init_speaker
    cfg = rcfg.v2()
    params, spk = init_params(cfg, seed=0), init_speaker(cfg, seed=0)
    with open(_tuning_file("f32_bf3")) as fh:
        tuning = json.load(fh)
    m = RAVE(cfg, params, spk, device=dev, precision="f32_bf3", tuning=tuning)
    ops = m.ops(ENCODE, B, T) + m.ops(DECODE, B, T // cfg.hop)
    # the pinned file covers every launch choice of both plans: nothing re-timed
    assert len(m.tuning()) == len(tuning)
    n_bf3 = sum(1 for o in ops if o["precision"] == N.PREC_BF16X3)
    n_coop = sum(1 for k, c, _ in tuning if k.startswith("unit|") and (int(c) >> 8))
    x = torch.from_numpy(synth_batch(B, T, 0)).to(dev)
    z = m.encode(x)
    y = m.decode(z)
    torch.cuda.synchronize()
    m.check()
    return dict(cfg=cfg, params=params, spk=spk, m=m, x=x, z=z, y=y, n_bf3=n_bf3, n_coop=n_coop)


def test_headline_plan_runs_bf16x3(headline):
    """The plan under test is the headline's arithmetic: bf16x3 units, C = 64
    residual stacks and convs, cooperative units at C = 512."""
    assert headline["n_bf3"] >= 28, headline["n_bf3"]
    assert headline["n_coop"] >= 4, headline["n_coop"]


@pytest.mark.parametrize("clip", [0, 11])
def test_headline_plan_vs_oracle(headline, clip):
    """Clips 0 and 11 of the timed batch: z and y against the float64 oracle."""
    from oracle.rave_oracle import Oracle
    h = headline
    o = Oracle(h["cfg"], h["params"], h["spk"], hk=h["m"].hk)
    xc = h["x"][clip:clip + 1].cpu().numpy()
    zr = o.encode(xc)
    ez = float(np.abs(h["z"][clip:clip + 1].cpu().numpy().astype(np.float64) - zr).max())
    yr = o.decode(zr)
    ey = float(np.abs(h["y"][clip:clip + 1].cpu().numpy().astype(np.float64) - yr).max())
    print(f"\n[parity] headline plan (f32_bf3, pinned, 16x65536) clip {clip} vs float64 oracle: "
          f"z {ez:.3e}, y {ey:.3e}")
    assert ez < TOL and ey < TOL


def test_headline_plan_batch_independence_and_determinism(headline):
    """Reruns of the pinned plan are bitwise equal; a clip run alone (its own
    B = 1 plan) matches its row of the batch."""
    h = headline
    m, x = h["m"], h["x"]
    y2 = m.decode(m.encode(x))
    y3 = m.forward(x[5:6].contiguous())
    torch.cuda.synchronize()
    m.check()
    assert torch.equal(h["y"], y2)
    assert torch.isfinite(y2).all()
    assert float((h["y"][5:6] - y3).abs().max()) < 1e-5


def test_exact_fp32_pinned_plan_vs_headline(headline, dev):
    """The exact-fp32 pinned plan (bench's ``f32_exact`` leg) on the same batch
    agrees with the headline within the north-star tolerance."""
    from rave_amd.model import RAVE
    h = headline
    with open(_tuning_file("f32_tuned")) as fh:
        tuning = json.load(fh)
    m = RAVE(h["cfg"], h["params"], h["spk"], device=dev, precision="f32_tuned", tuning=tuning)
    y = m.forward(h["x"])
    torch.cuda.synchronize()
    m.check()
    d = float((y - h["y"]).abs().max())
    print(f"\n[parity] headline vs exact-fp32 pinned plan, 16x65536: max-abs {d:.3e}")
    assert d < TOL
