"""``Resampler``: integer-ratio sample-rate conversion around the model
(rave/resampler.py:9-66; nn~ ``--sr``, scripts/export.py:101-106, 159-160,
303-304, 331-332).

For ``ratio = target_sr // model_sr`` the reference designs one Kaiser
lowpass ``h = kaiser_filter(pi / ratio, 140)`` (rave/pqmf.py:55-70) and uses it
twice through cached_conv convolutions:

* ``to_model_sampling_rate``: Conv1d(1, 1, len(h), stride=ratio,
  padding=get_padding(len(h), ratio)) -- decimation (:29-38);
* ``from_model_sampling_rate``: h left-padded to a multiple of ratio, split
  into its ``ratio`` polyphase rows (row p = h[p::ratio]), each left-padded to
  odd length, as Conv1d(1, ratio, K, padding=get_padding(K)); the (B, ratio, T)
  output is interleaved to (B, 1, ratio T) (:40-66).

Both run on ``rave_fir`` (csrc/speaker.hip), a polyphase FIR over a zero-padded
window: ``y[b, t*P + p] = sum_k h[p, k] x[b, t*stride + k - pad_left]``.
Streaming (cached_conv, ``streaming=True``) keeps each conv's input history
on the device, exactly as CachedConv1d does: the stream is delayed by
``stride_delay = (s - r % s) % s`` samples, then ``l + r`` samples of cache are
prepended, so every block of T inputs yields T / s outputs.
"""
from __future__ import annotations

import ctypes as C
from typing import Tuple

import numpy as np

from .config import get_padding

ATTENUATION = 140.0


def kaiser_filter(wc: float, atten: float) -> np.ndarray:
    """rave/pqmf.py:55-70 (``firwin(nyq=pi)`` is ``fs=2*pi``)."""
    from scipy.signal import firwin, kaiserord
    n_, beta = kaiserord(atten, wc / np.pi)
    n_ = 2 * (n_ // 2) + 1
    return firwin(n_, wc, window=("kaiser", beta), scale=False, fs=2 * np.pi)


def design(target_sr: int, model_sr: int) -> Tuple[int, np.ndarray, np.ndarray]:
    """(ratio, down (1, K_d) float32, up (ratio, K_u) float32) as
    Resampler.__init__ builds its two conv weights (rave/resampler.py:12-58)."""
    if target_sr == model_sr:
        raise ValueError("identical source and target rates")
    ratio = target_sr // model_sr
    if ratio < 2 or ratio * model_sr != target_sr:
        raise ValueError(f"target rate {target_sr} must be an integer multiple (>= 2) of {model_sr}")
    filt = kaiser_filter(np.pi / ratio, ATTENUATION).astype(np.float32)
    down = filt.reshape(1, -1)
    pad = len(filt) % ratio
    if (len(filt) + pad) % ratio:
        # the reference pads len(h) % ratio taps (rave/resampler.py:41-44), so its
        # reshape into `ratio` polyphase rows only succeeds for ratios 2 and 3
        raise ValueError(f"ratio {ratio}: the {len(filt)}-tap filter padded by {pad} does not split into "
                         f"{ratio} polyphase rows (rave/resampler.py:41-44)")
    up = np.pad(filt, (pad, 0)).reshape(-1, ratio).T
    pad = (up.shape[-1] + 1) % 2
    up = np.pad(up, ((0, 0), (pad, 0)))
    return ratio, np.ascontiguousarray(down), np.ascontiguousarray(up)


class _FirStage:
    """One cached_conv Conv1d(1, P, K, stride) on rave_fir, offline or cached."""

    def __init__(self, taps: np.ndarray, stride: int, causal: bool, streaming: bool, dev):
        import torch
        self.torch, self.dev = torch, dev
        self.taps = np.ascontiguousarray(taps, np.float32)
        self.h = None                                   # uploaded on first use
        self.phases, self.k = taps.shape
        self.stride = stride
        self.pad = get_padding(self.k, stride, causal=causal)
        self.streaming = streaming
        s, r = stride, self.pad[1]
        self.stride_delay = (s - (r % s)) % s          # CachedConv1d (cached_conv, restated)
        self.hist = self.pad[0] + self.pad[1] + self.stride_delay
        self.buf = None

    def reset(self):
        self.buf = None

    def __call__(self, x):
        """x (B, T) fp32 contiguous -> y (B, P * T_out)."""
        from . import _native as N
        torch = self.torch
        if self.h is None:
            self.h = torch.from_numpy(self.taps).to(self.dev)
        B, T = x.shape
        if not self.streaming:
            # F.pad(l, r) then conv: (T + l + r - K) // s + 1 outputs
            t_out = (T + self.pad[0] + self.pad[1] - self.k) // self.stride + 1
            src, sb, pad_left, t_in = x, x.stride(0), self.pad[0], T
        else:
            if T % self.stride:
                raise ValueError(f"block length {T} must be a multiple of the stride {self.stride}")
            t_out = T // self.stride
        y = torch.empty(B, self.phases * t_out, device=self.dev)
        if self.streaming:
            H = self.hist
            if self.buf is None or self.buf.shape != (B, H + T):
                self.buf = torch.zeros(B, H + T, device=self.dev)
            self.buf[:, H:].copy_(x)
            src, sb, pad_left, t_in = self.buf, self.buf.stride(0), 0, H + T
        a = N.FirArgs(batch=B, t_in=t_in, t_out=t_out, phases=self.phases, taps=self.k, stride=self.stride,
                      pad_left=pad_left, x=src.data_ptr(), x_sb=sb, y=y.data_ptr(), y_sb=y.stride(0),
                      h=self.h.data_ptr())
        N.check(N.lib.rave_fir(C.byref(a), C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)),
                "resampler fir")
        if self.streaming:
            # cache: the newest H samples of [history | block] become the next history
            H = self.hist
            self.buf[:, :H].copy_(self.buf[:, T:T + H].clone())
        return y


class Resampler:
    """Resampler(target_sr, model_sr) on the device.  ``causal`` is cached_conv's
    padding mode (causal.gin); ``streaming`` selects the cached (block by block)
    form with per-instance history."""

    def __init__(self, target_sr: int, model_sr: int, device=None, causal: bool = False,
                 streaming: bool = False):
        import torch
        ratio, down, up = design(target_sr, model_sr)
        if streaming and ratio % 2:
            # rave/resampler.py:22-25 (the reference's check is on odd ratios)
            raise ValueError(f"When using streaming mode, resampling ratio must be a power of 2, got {ratio}")
        self.ratio, self.model_sr, self.target_sr = ratio, model_sr, target_sr
        self.dev = torch.device(device or "cuda")
        self.down_taps, self.up_taps = down, up
        self._down = _FirStage(down, ratio, causal, streaming, self.dev)
        self._up = _FirStage(up, 1, causal, streaming, self.dev)

    def reset(self):
        self._down.reset()
        self._up.reset()

    @staticmethod
    def _check(x, name):
        if x.dim() != 3 or x.shape[1] != 1:
            raise ValueError(f"{name}: expected (B, 1, T), got {tuple(x.shape)}")

    def to_model_sampling_rate(self, x):
        """(B, 1, T) at target_sr -> (B, 1, T / ratio) at model_sr (rave/resampler.py:60-61)."""
        self._check(x, "to_model_sampling_rate")
        return self._down(x[:, 0].contiguous()).unsqueeze(1)

    def from_model_sampling_rate(self, x):
        """(B, 1, T) at model_sr -> (B, 1, ratio T) at target_sr (rave/resampler.py:63-66)."""
        self._check(x, "from_model_sampling_rate")
        return self._up(x[:, 0].contiguous()).unsqueeze(1)
