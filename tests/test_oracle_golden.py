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


def adain_sequence(g):
    """(tag, learn_x, learn_y, x) of the AdaIN fixture's call sequence."""
    flags = {"learn_y": (False, True), "learn_x": (True, False), "transfer": (False, False),
             "learn_x_bs1": (True, False)}
    xs = {"learn_y": g["x_tgt"], "learn_x": g["x_src"], "transfer": g["x_src"],
          "learn_x_bs1": g["x_src"][:1]}
    return [(str(t),) + flags[str(t)] + (xs[str(t)],) for t in g["steps"]]


@pytest.mark.parametrize("name,cfg", [("v3_adain_small", rcfg.v3(capacity=8)),
                                      ("v3_adain", rcfg.v3())])
def test_adain_style_transfer(golden, name, cfg):
    """learn_y -> learn_x -> transfer -> learn_x(bs=1), buffers updated in place."""
    from rave_amd.graph import build_graph
    g = golden(name)
    o = _oracle(cfg, g)
    mods = build_graph(cfg).adain_modules
    assert [n for n, _ in mods] == [str(n) for n in g["names"]]
    o.adain_stats = Oracle.fresh_adain_state(mods)
    for i, (tag, lx, ly, x) in enumerate(adain_sequence(g)):
        o.learn_x, o.learn_y = lx, ly
        z = o.encode(x)
        assert rel(z, g[f"step{i}/z"]) < TOL, tag
        y = o.decode(z)
        assert maxabs(y, g[f"step{i}/y"]) < TOL, tag
    for n, _ in mods:
        st = o.adain_stats[n]
        for b in ("mean_x", "std_x", "mean_y", "std_y"):
            assert rel(st[b], g[f"final/{n}.{b}"]) < 1e-4, (n, b)
        assert st["num_update_x"] == float(g[f"final/{n}.num_update_x"][0])
        assert st["num_update_y"] == float(g[f"final/{n}.num_update_y"][0])


def test_manifest_covers_every_fixture():
    """Provenance: every committed fixture is listed in MANIFEST.json with the
    sha256 prefix make_golden.py recorded when the reference produced it."""
    import hashlib
    import json
    import os
    d = os.path.join(os.path.dirname(__file__), "golden")
    with open(os.path.join(d, "MANIFEST.json")) as fh:
        files = json.load(fh)["files"]
    npz = sorted(f for f in os.listdir(d) if f.endswith(".npz"))
    assert sorted(files) == npz
    for f in npz:
        with open(os.path.join(d, f), "rb") as fh:
            assert hashlib.sha256(fh.read()).hexdigest()[:16] == files[f], f
