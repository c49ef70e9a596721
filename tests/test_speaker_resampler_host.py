"""SpeakerRAVE and Resampler on the CPU: the oracle against the reference's
own outputs (tests/golden/speaker.npz, resampler.npz from make_golden.py),
and the host-side parts of rave_amd.speaker / rave_amd.resampler (filter
design, parameter folds, checkpoint loading, argument validation)."""
import ctypes as C

import numpy as np
import pytest

from oracle import speaker_oracle as so
from rave_amd import resampler as R
from rave_amd import speaker as S


def maxabs(a, b):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max())


@pytest.mark.parametrize("mode", ["centered", "causal"])
def test_speaker_oracle_golden(golden, mode):
    g = golden("speaker")
    p = S.init_params(int(g["seed"]))
    trace = {}
    emb = so.speaker_forward(p, g[f"{mode}/bands"], causal=mode == "causal", trace=trace)
    assert emb.shape == (2, 256)
    assert maxabs(emb, g[f"{mode}/emb"]) < 1e-5
    for name in ("layer2", "layer3", "layer4", "cat_layer", "out_layer"):
        ref = g[f"{mode}/{name}"]
        assert maxabs(trace[name], ref) / max(1.0, float(np.abs(ref).max())) < 1e-5, name


def test_speaker_head_fold_equals_unfolded(golden):
    """The host folds (BN into neighbours, time-constant attention columns into
    a per-clip bias) give the same pooled embedding as the oracle's unfolded head."""
    g = golden("speaker")
    p = S.init_params(0)
    rng = np.random.default_rng(3)
    x = rng.standard_normal((2, 768, 40))                         # out_layer output (pre-act)
    h = S.fold_head(p)
    a = np.where(x > 0, x, 0.2 * x)
    mean, std = a.mean(-1), np.sqrt(np.clip(a.var(-1, ddof=1), 1e-4, 1e4))
    bias = h["att0_b"][None] + np.concatenate([mean, std], 1) @ h["att0_stat"].T.astype(np.float64)
    hid = np.einsum("oi,bit->bot", h["att0_x"][:, :, 0], a) + bias[:, :, None]
    lg = np.einsum("oi,bit->bot", h["att3_w"][:, :, 0], np.maximum(hid, 0)) + h["att3_b"][None, :, None]
    w = np.exp(lg - lg.max(-1, keepdims=True))
    w /= w.sum(-1, keepdims=True)
    mu = (a * w).sum(-1)
    sg = np.sqrt(np.clip((a * a * w).sum(-1) - mu ** 2, 1e-4, 1e4))
    y = np.concatenate([mu, sg], 1) @ h["fc_w"].T.astype(np.float64) + h["fc_b"]
    # the unfolded reference head on the same out_layer activations
    g_x = np.concatenate([a, np.repeat(mean[..., None], 40, -1), np.repeat(std[..., None], 40, -1)], 1)
    hh = np.einsum("oi,bit->bot", p["attention.0.weight"][:, :, 0], g_x) + p["attention.0.bias"][None, :, None]
    hh = so._bn(p, "attention.2", np.maximum(hh, 0))
    l2 = np.einsum("oi,bit->bot", p["attention.3.weight"][:, :, 0], hh) + p["attention.3.bias"][None, :, None]
    w2 = np.exp(l2 - l2.max(-1, keepdims=True))
    w2 /= w2.sum(-1, keepdims=True)
    mu2 = (a * w2).sum(-1)
    sg2 = np.sqrt(np.clip((a * a * w2).sum(-1) - mu2 ** 2, 1e-4, 1e4))
    y2 = so._bn(p, "bn5", np.concatenate([mu2, sg2], 1)) @ p["fc6.weight"].T + p["fc6.bias"]
    assert maxabs(y, y2) < 1e-5


def test_speaker_load_state_like_load_speaker_statedict():
    """rave/model.py:278-300: '__S__.' prefixes dropped, pqmf entries set aside;
    unused entries (bn6, num_batches_tracked) ignored; missing/misshaped raise."""
    p = S.init_params(1)
    ckpt = {"__S__." + k: v for k, v in p.items()}
    ckpt["__S__.pqmf.hk"] = np.zeros((16, 512), np.float32)
    ckpt["__S__.bn6.weight"] = np.ones(256, np.float32)
    ckpt["__S__.bn5.num_batches_tracked"] = np.array(3)
    out = S.load_state(ckpt)
    assert set(out) == set(S.param_shapes())
    assert all(np.array_equal(out[k], p[k]) for k in p)
    bad = dict(ckpt)
    del bad["__S__.fc6.bias"]
    with pytest.raises(KeyError):
        S.load_state(bad)
    bad = dict(ckpt)
    bad["__S__.fc6.bias"] = np.zeros(3, np.float32)
    with pytest.raises(ValueError):
        S.load_state(bad)


@pytest.mark.parametrize("ratio,mode", [(2, "centered"), (3, "centered"), (2, "causal")])
def test_resampler_design_and_oracle_golden(golden, ratio, mode):
    g = golden("resampler")
    key = f"r{ratio}_{mode}"
    r, down, up = R.design(48000 * ratio, 48000)
    assert r == ratio
    assert np.array_equal(down, g[f"{key}/down_w"][0])          # bit-exact filter design
    assert np.array_equal(up, g[f"{key}/up_w"][:, 0])
    c = mode == "causal"
    assert maxabs(so.resampler_down(g["x"], ratio, c), g[f"{key}/down"]) < 2e-6
    assert maxabs(so.resampler_up(g["x"], ratio, c), g[f"{key}/up"]) < 2e-6


@pytest.mark.parametrize("mode", ["centered", "causal"])
def test_resampler_stream_oracle_golden(golden, mode):
    g = golden("resampler")
    xs = g["stream/x"]
    blocks = [xs[..., i * 2048:(i + 1) * 2048] for i in range(xs.shape[-1] // 2048)]
    for d in ("down", "up"):
        y = np.concatenate(so.resampler_stream(blocks, 2, mode == "causal", d), -1)
        assert maxabs(y, g[f"stream/r2_{mode}/{d}"]) < 2e-6


def test_resampler_rejects_what_the_reference_rejects():
    with pytest.raises(ValueError):
        R.design(48000, 48000)                 # identical rates (rave/resampler.py:14)
    with pytest.raises(ValueError):
        R.design(96000 + 1, 48000)             # not an integer ratio (:19-20)
    for ratio in range(4, 9):                  # the reference's polyphase reshape fails (:41-44)
        with pytest.raises(ValueError):
            R.design(48000 * ratio, 48000)


def test_edge_kernels_validate_arguments():
    from rave_amd import _native as N
    a = N.FirArgs(batch=1, t_in=16, t_out=8, phases=1, taps=5, stride=2, pad_left=2)
    assert N.lib.rave_fir(C.byref(a), None) == N.RAVE_ERR_ARG          # null pointers
    a = N.FirArgs(batch=1, t_in=16, t_out=8, phases=8, taps=1000, stride=1, x=8, y=8, h=8, y_sb=64)
    assert N.lib.rave_fir(C.byref(a), None) == N.RAVE_ERR_ARG          # taps x phases too large
    r = N.RowStatsArgs(batch=1, channels=4, t_len=8, act=N.ACT["snake"], x=8, y=8, y_sb=8)
    assert N.lib.rave_row_stats(C.byref(r), None) == N.RAVE_ERR_ARG     # snake not supported here
    r = N.RowStatsArgs(batch=1, channels=4, t_len=8, act=0, x=8, y=8, y_sb=4)
    assert N.lib.rave_row_stats(C.byref(r), None) == N.RAVE_ERR_ARG     # overlapping output rows
    ln = N.LinearArgs(batch=1, n_in=0, n_out=4, x=8, w=8, y=8)
    assert N.lib.rave_linear(C.byref(ln), None) == N.RAVE_ERR_ARG
    mp = N.MaxPoolArgs(batch=1, channels=1, t_out=0, kernel=2, x=8, y=8)
    assert N.lib.rave_maxpool(C.byref(mp), None) == N.RAVE_ERR_ARG
