"""PQMF filter design (init-time, host) -- restates rave/pqmf.py.

* ``kaiser_filter`` rave/pqmf.py:55-70, ``loss_wc`` :73-80, ``get_prototype``
  :83-89 (Nelder-Mead on the cutoff; scipy ``firwin(nyq=pi)`` is ``fs=2*pi``).
* ``get_qmf_bank`` :32-52 cosine modulation; ``center_pad_next_pow_2`` :20-23;
  ``make_odd`` :26-29; the analysis kernel ``hkf`` and the polyphase synthesis
  kernel ``hki`` of ``CachedPQMF.__init__`` :236-263.

Only the coefficients are computed here; filtering runs in the HIP kernels
(rave_amd/csrc/pqmf.hip).  Parity of ``hk`` with the reference is pinned by
tests/golden/pqmf.npz (sha256[:16] of hk = 4d86cced7ee86762).
"""
from __future__ import annotations

import functools
import math
from typing import Tuple

import numpy as np


def _kaiser(wc: float, atten: float, N=None) -> np.ndarray:
    from scipy.signal import firwin, kaiserord
    n_, beta = kaiserord(atten, wc / np.pi)
    n_ = 2 * (n_ // 2) + 1
    return firwin(N if N is not None else n_, wc, window=("kaiser", beta), scale=False, fs=2 * np.pi)


def _objective(wc, atten, M, N):
    h = _kaiser(float(np.asarray(wc).reshape(-1)[0]), atten, N)
    g = np.convolve(h, h[::-1], "full")
    return np.max(np.abs(g[g.shape[-1] // 2::2 * M][1:]))


@functools.lru_cache(maxsize=8)
def design_bank(attenuation: float = 100.0, n_band: int = 16) -> np.ndarray:
    """hk (n_band, next_pow2(N)) float32, as CachedPQMF registers it."""
    from scipy.optimize import fmin
    wc = fmin(lambda w: _objective(w, attenuation, n_band, None), 1 / n_band, disp=0)[0]
    # get_qmf_bank (rave/pqmf.py:32-52) runs on torch int64 / float32 CPU
    # tensors: the modulation argument, the cosine and 2*h*mod are float32
    # operations, so they are evaluated with the same torch ops (bit-exact with
    # the reference's hk, tests/test_host.py); float64 differs by ~1.7e-7.
    import torch
    h = torch.from_numpy(_kaiser(wc, attenuation)).float()
    N = h.shape[-1]
    k = torch.arange(n_band).reshape(-1, 1)
    t = torch.arange(-(N // 2), N // 2 + 1)
    phase = (-1) ** k * math.pi / 4
    mod = torch.cos((2 * k + 1) * math.pi / (2 * n_band) * t + phase)
    hk = (2 * h * mod).numpy()
    pad = 2 ** math.ceil(math.log2(N)) - N
    return np.pad(hk, ((0, 0), (pad // 2, pad // 2 + pad % 2)))


def kernels(hk: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """(hkf (n_band, taps_a), hki (n_band, n_band, taps_s)) float32."""
    m, L = hk.shape
    hkf = np.pad(hk, ((0, 0), (0, 1))) if L % 2 == 0 else hk
    hki = hk[:, ::-1].reshape(m, L // m, m).transpose(2, 0, 1)
    if hki.shape[-1] % 2 == 0:
        hki = np.pad(hki, ((0, 0), (0, 0), (0, 1)))
    return np.ascontiguousarray(hkf, np.float32), np.ascontiguousarray(hki, np.float32)
