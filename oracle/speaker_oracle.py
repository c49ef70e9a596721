"""CPU ORACLE for SpeakerRAVE and the Resampler -- TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module (as the checker).  The product path
(rave_amd.speaker / rave_amd.resampler) never imports it.

Plain float64 numpy restatement, written from the reference read as text:

* ``speaker_forward`` -- SpeakerRAVE.forward, rave/CombinedRave.py:301-328,
  layers :200-299 (identity normalization :18-24, DilatedUnit :79-108,
  Residual :27-41), torch.var unbiased, BatchNorm1d eval (eps 1e-5),
  Softmax over time.
* ``resampler_*`` -- rave/resampler.py:9-66 with cached_conv's Conv1d padding
  (non-cached: F.pad then conv; cached: ``stride_delay`` crop-pad + ``l + r``
  cache, as tests/golden/refshim/cached_conv.py restates it).

Pinned by tests/test_oracle_golden.py against tests/golden/speaker.npz and
tests/golden/resampler.npz, produced by running the reference modules
(tests/golden/make_golden.py ``gen_speaker`` / ``gen_resampler``).
"""
from __future__ import annotations

from typing import Mapping

import numpy as np

from .rave_oracle import conv1d, get_padding, kaiser_filter, leaky_relu

F64 = np.float64


def _conv(p, name, x, k, stride=1, dilation=1, causal=False):
    pad = get_padding(k, stride, dilation, causal)
    return conv1d(x, np.asarray(p[name + ".weight"], F64), p[name + ".bias"], stride, dilation, pad)


def _unit(p, prefix, x, d, causal):
    """Residual(DilatedUnit(dim, 3, d)) with LeakyReLU(.2) (rave/CombinedRave.py:79-108)."""
    u = f"{prefix}.0.aligned.branches.0.net"
    h = _conv(p, u + ".1", leaky_relu(x), 3, 1, d, causal)
    return x + _conv(p, u + ".3", leaky_relu(h), 1)


def _bn(p, name, x):
    s = np.asarray(p[name + ".weight"], F64) / np.sqrt(np.asarray(p[name + ".running_var"], F64) + 1e-5)
    t = np.asarray(p[name + ".bias"], F64) - s * np.asarray(p[name + ".running_mean"], F64)
    shape = (1, -1) + (1,) * (x.ndim - 2)
    return x * s.reshape(shape) + t.reshape(shape)


def speaker_forward(p: Mapping[str, np.ndarray], bands: np.ndarray, causal: bool = False,
                    trace: dict = None) -> np.ndarray:
    """(B, 16, T) PQMF bands -> (B, 256) embedding (rave/CombinedRave.py:301-328)."""
    x = np.asarray(bands, F64)
    x = _conv(p, "in_layer", x, 7, causal=causal)
    outs = []
    for name, k, s, d in (("layer2", 8, 4, 1), ("layer3", 8, 4, 3), ("layer4", 4, 2, 5)):
        x = _unit(p, name, x, d, causal)
        x = _conv(p, name + ".2", leaky_relu(x), k, s, causal=causal)
        outs.append(x)
    x2, x3 = outs[1], outs[2]
    x4 = _conv(p, "cat_layer", x3, 1)
    B, C, T2 = x2.shape
    mp = x2[..., : (T2 // 2) * 2].reshape(B, C, T2 // 2, 2).max(-1)          # MaxPool1d(2)
    x = np.concatenate([mp, x3, x4], 1)
    xo = _conv(p, "out_layer", x, 3, causal=causal)
    if trace is not None:        # module outputs, as forward hooks see them
        trace.update(layer2=outs[0], layer3=x2, layer4=x3, cat_layer=x4, out_layer=xo)
    x = leaky_relu(xo)
    t = x.shape[-1]
    mean = x.mean(-1, keepdims=True)
    std = np.sqrt(np.clip(x.var(-1, ddof=1, keepdims=True), 1e-4, 1e4))
    g = np.concatenate([x, np.repeat(mean, t, -1), np.repeat(std, t, -1)], 1)
    h = conv1d(g, np.asarray(p["attention.0.weight"], F64), p["attention.0.bias"])
    h = _bn(p, "attention.2", np.maximum(h, 0.0))
    a = conv1d(h, np.asarray(p["attention.3.weight"], F64), p["attention.3.bias"])
    a = np.exp(a - a.max(-1, keepdims=True))
    w = a / a.sum(-1, keepdims=True)
    mu = (x * w).sum(-1)
    sg = np.sqrt(np.clip((x ** 2 * w).sum(-1) - mu ** 2, 1e-4, 1e4))
    v = _bn(p, "bn5", np.concatenate([mu, sg], 1))
    return v @ np.asarray(p["fc6.weight"], F64).T + np.asarray(p["fc6.bias"], F64)


# ------------------------------------------------------------------ Resampler
def resampler_filters(ratio: int):
    """(down (1,1,K), up (ratio,1,K')) float32 as rave/resampler.py:27-58 builds them."""
    filt = kaiser_filter(np.pi / ratio, 140).astype(np.float32)
    pad = len(filt) % ratio
    up = np.pad(filt, (pad, 0)).reshape(-1, ratio).T
    up = np.pad(up, ((0, 0), ((up.shape[-1] + 1) % 2, 0)))
    return filt.reshape(1, 1, -1), np.ascontiguousarray(up[:, None, :])


def resampler_down(x: np.ndarray, ratio: int, causal: bool = False) -> np.ndarray:
    """to_model_sampling_rate, non-cached (rave/resampler.py:60-61)."""
    down, _ = resampler_filters(ratio)
    k = down.shape[-1]
    return conv1d(x, down.astype(F64), None, ratio, 1, get_padding(k, ratio, 1, causal))


def resampler_up(x: np.ndarray, ratio: int, causal: bool = False) -> np.ndarray:
    """from_model_sampling_rate, non-cached (rave/resampler.py:63-66)."""
    _, up = resampler_filters(ratio)
    k = up.shape[-1]
    y = conv1d(x, up.astype(F64), None, 1, 1, get_padding(k, 1, 1, causal))   # (B, ratio, T)
    return y.transpose(0, 2, 1).reshape(y.shape[0], 1, -1)


def _cached_conv_stream(x_blocks, w, stride, pad):
    """CachedConv1d over consecutive blocks (cached_conv restated): the input is
    delayed by stride_delay samples, then l + r samples of cache are prepended."""
    l, r = pad
    sd = (stride - (r % stride)) % stride
    hist = np.zeros((x_blocks[0].shape[0], x_blocks[0].shape[1], l + r + sd))
    outs = []
    for xb in x_blocks:
        buf = np.concatenate([hist, np.asarray(xb, F64)], -1)
        T = xb.shape[-1]
        win = buf[..., : buf.shape[-1] - sd] if sd else buf
        outs.append(conv1d(win, w, None, stride, 1, (0, 0)))
        hist = buf[..., T:]
    return outs


def resampler_stream(blocks, ratio: int, causal: bool, direction: str):
    """Cached (streaming) to/from_model_sampling_rate over a list of (B, 1, T) blocks."""
    down, up = resampler_filters(ratio)
    if direction == "down":
        k = down.shape[-1]
        return _cached_conv_stream(blocks, down.astype(F64), ratio, get_padding(k, ratio, 1, causal))
    k = up.shape[-1]
    ys = _cached_conv_stream(blocks, up.astype(F64), 1, get_padding(k, 1, 1, causal))
    return [y.transpose(0, 2, 1).reshape(y.shape[0], 1, -1) for y in ys]
