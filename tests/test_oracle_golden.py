"""The CPU oracle (oracle/rave_oracle.py) against the golden fixtures produced
by running the reference itself (tests/golden/make_golden.py).  This is what
pins the oracle before the HIP path is compared to it."""
import numpy as np
import pytest

from oracle.rave_oracle import Oracle, pqmf_filters, qmf_bank
from rave_amd import config as rcfg
from rave_amd.weights import init_params

TOL = 1e-4   # north star: <= 1e-4 max-abs vs the reference fp32 CPU path


def maxabs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


def rel(a, b):
    """max-abs error scaled by max(1, max|b|) (fp32 reference vs float64 oracle)."""
    return maxabs(a, b) / max(1.0, float(np.abs(b).max()))


def test_pqmf_bank(golden):
    g = golden("pqmf")
    hk = qmf_bank(100, 16)
    assert hk.shape == (16, 512)
    assert maxabs(hk, g["hk"]) < 1e-6


@pytest.mark.parametrize("causal", [False, True])
def test_pqmf_analysis_synthesis(golden, causal):
    g = golden("pqmf")
    mode = "causal" if causal else "centered"
    o = Oracle(rcfg.v2(causal=causal), {}, np.zeros(256), hk=g["hk"])
    assert rel(o.pqmf_analysis(g["x"]), g[f"analysis_{mode}"]) < 1e-5
    assert rel(o.pqmf_synthesis(g["bands"]), g[f"synthesis_{mode}"]) < 1e-5
    assert rel(o.pqmf_synthesis(o.pqmf_analysis(g["x"])), g[f"roundtrip_{mode}"]) < 1e-5


def _oracle(cfg, g):
    return Oracle(cfg, init_params(cfg, seed=int(g["seed"])), g["speaker"], hk=golden_hk())


_HK = {}


def golden_hk():
    if "hk" not in _HK:
        import os
        from tests.conftest import GOLDEN
        _HK["hk"] = np.load(os.path.join(GOLDEN, "pqmf.npz"))["hk"]
    return _HK["hk"]


@pytest.mark.parametrize("name,cfg", [("v2", rcfg.v2()), ("causal", rcfg.causal())])
def test_v2_end_to_end(golden, name, cfg):
    g = golden(name)
    o = _oracle(cfg, g)
    z = o.encode(g["x"])
    assert maxabs(z, g["z"]) < TOL
    y = o.decode(g["z"])
    assert maxabs(y, g["y"]) < TOL


@pytest.mark.parametrize("name,cfg", [("v2_small_layers", rcfg.v2(capacity=8)),
                                      ("v3_noise_small_layers", rcfg.v3_noise(capacity=8))])
def test_per_layer(golden, name, cfg):
    g = golden(name)
    o = _oracle(cfg, g)
    o.record = True
    y = o.forward(g["x"], g.get("noise_u"))
    assert maxabs(y, g["y"]) < TOL
    layers = [k for k in g if k.startswith("layer/")]
    assert len(layers) >= 40
    for k in layers:
        assert maxabs(o.trace[k[6:]], g[k]) < TOL, k


def test_discrete(golden):
    g = golden("discrete")
    cfg = rcfg.discrete()
    o = _oracle(cfg, g)
    ze = o.encode(g["x"])
    assert maxabs(ze, g["z_enc"]) < TOL
    idx = o.rvq_encode(g["z_enc"])
    assert (idx == g["rvq_idx"]).all()
    zq = o.rvq_decode(g["rvq_idx"])
    assert maxabs(zq, g["z_q"]) < TOL
    assert maxabs(o.decode(g["z"]), g["y"]) < TOL


def test_rvq(golden):
    g = golden("rvq")
    cfg = rcfg.discrete()
    o = Oracle(cfg, init_params(cfg, seed=int(g["seed"])), np.zeros(256), hk=golden_hk())
    idx, gaps = o.rvq_encode(g["z"], return_gaps=True)
    assert (idx == g["idx"]).all()
    assert maxabs(o.rvq_decode(g["idx"]), g["zq"]) < TOL


def test_v3_noise(golden):
    g = golden("v3_noise")
    o = _oracle(rcfg.v3_noise(), g)
    assert maxabs(o.encode(g["x"]), g["z"]) < TOL
    assert maxabs(o.decode(g["z"], g["noise_u"]), g["y"]) < TOL


def test_causal_streaming_is_delayed_oneshot(golden):
    """Reference streaming decode == one-shot causal decode delayed by 928
    samples (four ConvTranspose1d r//2 delays: 32+16+8+2 band frames) once
    the left receptive field has filled (the cached ConvTranspose1d emits the
    r//2 leading samples one-shot mode crops, so the first ~9.5k samples are a
    start-up transient)."""
    g = golden("causal_stream")
    d, warm = 928, 10240
    ys, yo = g["y_stream"][..., d:], g["y_oneshot"][..., :-d]
    assert maxabs(ys[..., warm:], yo[..., warm:]) < 1e-5
    assert maxabs(g["z_stream"], g["z_oneshot"]) < 1e-5
    o = _oracle(rcfg.causal(), g)
    assert maxabs(o.decode(g["z"]), g["y_oneshot"]) < TOL
