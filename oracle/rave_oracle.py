"""CPU ORACLE for the RAVE encode->decode path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The
product path (rave_amd) never imports it and has no CPU fallback.

A plain-numpy (float64) restatement of the reference algorithm, written from
the reference source read as text:

* PQMF design/analysis/synthesis -- rave/pqmf.py:13-29 (reverse_half,
  center_pad_next_pow_2, make_odd), :32-52 (get_qmf_bank), :55-89
  (kaiser_filter, loss_wc, get_prototype), :234-284 (CachedPQMF forward /
  inverse with cc.get_padding(513) / get_padding(33)).
* Conv / ConvTranspose semantics of cached_conv in non-cached mode (explicit
  F.pad then conv; ConvTranspose1d padding r//2) -- the third-party package
  ``cached-conv>=2.5.0`` (requirements.txt:14, unpinned, absent here);
  restated from its published behaviour.
* DilatedUnit / Residual -- rave/blocks.py:32-46, 84-113; EncoderV2
  rave/blocks.py:508-597; GeneratorV2 rave/blocks.py:600-710;
  LeakyReLU(.2); Snake rave/blocks.py:845-853; AdaIN (eval identity unless
  stats are given) rave/blocks.py:856-919.
* RAVE.encode/decode/forward -- rave/model.py:594-634 (6 of 16 bands, constant
  speaker concat, no reparametrize).
* RVQ encode/decode -- rave/quantization.py:131-140, 239-249, 302-318.
* NoiseGeneratorV2 -- rave/blocks.py:244-291 with mod_sigmoid
  rave/core.py:66-67, amp_to_impulse_response :95-116, fft_convolve :119-129;
  the uniform noise tensor is an explicit input (``torch.rand_like`` at
  rave/blocks.py:287 is not reproducible).

Parity pinned: tests/test_oracle_golden.py checks every function here against
the fixtures in tests/golden/ produced by running the reference itself
(tests/golden/make_golden.py).  The one reference behaviour no reference test
pins is cached_conv's centred even-kernel split ((p-1)//2, p//2); the fixtures
were produced with that choice.
"""
from __future__ import annotations

import math
from typing import Dict, Mapping, Optional, Sequence, Tuple

import numpy as np

F64 = np.float64


# =============================================================== PQMF design
def kaiser_filter(wc: float, atten: float, N: Optional[int] = None) -> np.ndarray:
    """rave/pqmf.py:55-70 (firwin with nyq=pi == fs=2*pi)."""
    from scipy.signal import firwin, kaiserord
    N_, beta = kaiserord(atten, wc / np.pi)
    N_ = 2 * (N_ // 2) + 1
    N = N if N is not None else N_
    return firwin(N, wc, window=("kaiser", beta), scale=False, fs=2 * np.pi)


def loss_wc(wc, atten, M, N):
    """rave/pqmf.py:73-80."""
    h = kaiser_filter(wc, atten, N)
    g = np.convolve(h, h[::-1], "full")
    g = np.abs(g[g.shape[-1] // 2::2 * M][1:])
    return np.max(g)


def get_prototype(atten: float, M: int, N: Optional[int] = None) -> np.ndarray:
    """rave/pqmf.py:83-89 (Nelder-Mead on the cutoff)."""
    from scipy.optimize import fmin
    wc = fmin(lambda w: loss_wc(w, atten, M, N), 1 / M, disp=0)[0]
    return kaiser_filter(wc, atten, N)


def qmf_bank(atten: float = 100.0, n_band: int = 16) -> np.ndarray:
    """hk (n_band, 2**ceil(log2 N)) as CachedPQMF registers it (fp32 math as
    the reference: prototype cast to float32, rave/pqmf.py:200-204)."""
    h = get_prototype(atten, n_band).astype(np.float32)
    N = h.shape[-1]
    k = np.arange(n_band).reshape(-1, 1)
    t = np.arange(-(N // 2), N // 2 + 1)
    p = ((-1.0) ** k) * math.pi / 4
    mod = np.cos((2 * k + 1) * math.pi / (2 * n_band) * t + p).astype(np.float32)
    hk = (2 * h * mod).astype(np.float32)
    nxt = 2 ** math.ceil(math.log2(hk.shape[-1]))
    pad = nxt - hk.shape[-1]
    return np.pad(hk, ((0, 0), (pad // 2, pad // 2 + pad % 2)))


def pqmf_filters(hk: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Analysis kernel (n_band, 1, K+1) and synthesis kernel (m, c, T/m + 1)
    of CachedPQMF.__init__ (rave/pqmf.py:236-263)."""
    m = hk.shape[0]
    hkf = np.pad(hk, ((0, 0), (0, 1)))[:, None, :] if hk.shape[-1] % 2 == 0 else hk[:, None, :]
    flip = hk[:, ::-1]
    tlen = hk.shape[-1] // m
    hki = flip.reshape(m, tlen, m).transpose(2, 0, 1)  # "c (t m) -> m c t"
    if hki.shape[-1] % 2 == 0:
        hki = np.pad(hki, ((0, 0), (0, 0), (0, 1)))
    return np.ascontiguousarray(hkf), np.ascontiguousarray(hki)


def get_padding(k: int, stride: int = 1, dilation: int = 1, causal: bool = False):
    if k == 1:
        return (0, 0)
    p = (k - 1) * dilation + 1
    return (p - 1, 0) if causal else ((p - 1) // 2, p // 2)


def reverse_half(x: np.ndarray) -> np.ndarray:
    """rave/pqmf.py:13-17: negate odd bands at even time indices."""
    y = np.array(x, copy=True)
    y[..., 1::2, ::2] *= -1
    return y


# =============================================================== conv primitives
def conv1d(x: np.ndarray, w: np.ndarray, b: Optional[np.ndarray] = None, stride: int = 1,
           dilation: int = 1, pad: Tuple[int, int] = (0, 0)) -> np.ndarray:
    """F.pad(x, pad) then F.conv1d, float64 im2col + matmul."""
    x = np.pad(np.asarray(x, F64), ((0, 0), (0, 0), pad))
    B, C, T = x.shape
    Co, Ci, K = w.shape
    assert Ci == C, (w.shape, x.shape)
    span = (K - 1) * dilation + 1
    To = (T - span) // stride + 1
    sb, sc, st = x.strides
    cols = np.lib.stride_tricks.as_strided(
        x, shape=(B, C, K, To), strides=(sb, sc, st * dilation, st * stride))
    y = np.einsum("ock,bckt->bot", np.asarray(w, F64), cols, optimize=True)
    if b is not None:
        y += np.asarray(b, F64)[None, :, None]
    return y


def conv_transpose1d(x: np.ndarray, w: np.ndarray, stride: int, padding: int,
                     b: Optional[np.ndarray] = None) -> np.ndarray:
    """nn.ConvTranspose1d(C_in, C_out, K, stride, padding); w (C_in, C_out, K)."""
    x = np.asarray(x, F64)
    B, Ci, T = x.shape
    _, Co, K = w.shape
    full = np.zeros((B, Co, (T - 1) * stride + K), F64)
    for k in range(K):
        contrib = np.einsum("io,bit->bot", np.asarray(w[:, :, k], F64), x, optimize=True)
        full[:, :, k:k + (T - 1) * stride + 1:stride] += contrib
    y = full[:, :, padding:full.shape[-1] - padding]
    if b is not None:
        y = y + np.asarray(b, F64)[None, :, None]
    return y


def leaky_relu(x, slope=0.2):
    return np.where(x > 0, x, x * slope)


def snake(x, alpha):
    """rave/blocks.py:852-853: x + (alpha+1e-9)^-1 * sin(alpha x)^2."""
    a = np.asarray(alpha, F64).reshape(1, -1, 1)
    return x + (1.0 / (a + 1e-9)) * np.sin(a * x) ** 2


def fold_wn(g, v):
    v = np.asarray(v, F64)
    n = np.sqrt((v.reshape(v.shape[0], -1) ** 2).sum(1))
    shape = (v.shape[0],) + (1,) * (v.ndim - 1)
    return v * (np.asarray(g, F64).reshape(shape) / n.reshape(shape))


# =============================================================== model restatement
class Oracle:
    """RAVE encode/decode over a reference-named parameter dict."""

    def __init__(self, cfg, params: Mapping[str, np.ndarray], speaker: np.ndarray,
                 hk: Optional[np.ndarray] = None, adain_stats: Optional[Mapping] = None):
        self.cfg = cfg
        self.p = params
        self.speaker = np.asarray(speaker, F64)
        self.hk = qmf_bank(cfg.pqmf_attenuation, cfg.n_band) if hk is None else np.asarray(hk, np.float32)
        self.hkf, self.hki = pqmf_filters(self.hk)
        self.adain_stats = adain_stats or {}
        self.learn_x = False
        self.learn_y = False
        self.trace: Dict[str, np.ndarray] = {}
        self.record = False

    # -------------------------------------------------------------- helpers
    def _w(self, name, wn=True):
        if wn:
            return fold_wn(self.p[name + ".weight_g"], self.p[name + ".weight_v"])
        return np.asarray(self.p[name + ".weight"], F64)

    def _b(self, name):
        return self.p.get(name + ".bias")

    def _act(self, x, module):
        if self.cfg.activation == "snake":
            return snake(x, self.p[module + ".alpha"])
        return leaky_relu(x, self.cfg.leaky_slope)

    def _conv(self, x, name, k, stride=1, dilation=1, wn=True, pad=None):
        if pad is None:
            pad = get_padding(k, stride, dilation, self.cfg.causal)
        y = conv1d(x, self._w(name, wn), self._b(name), stride, dilation, pad)
        if self.record:
            self.trace[name] = y
        return y

    def _adain(self, x, name):
        """AdaptiveInstanceNormalization.forward, eval mode (rave/blocks.py:896-919).

        ``adain_stats[name]`` holds the module's buffers (mean_x, std_x, mean_y,
        std_y: (MAX_BATCH, C, 1); num_update_x/y) and is updated in place like
        the reference's; ``self.learn_x`` / ``self.learn_y`` are the learn flags
        (set on every module at once, as nn~'s attributes do).  Without state
        the module is the identity."""
        st = self.adain_stats.get(name)
        if st is None:
            return x
        bs = x.shape[0]

        def update(key, src, count):
            tgt = st[key]
            tgt[:bs] = tgt[:bs] + (src - tgt[:bs]) / (count + 1)

        if self.learn_y:
            n = float(st.get("num_update_y", 0.0))
            update("mean_y", x.mean(-1, keepdims=True), n)
            update("std_y", x.std(-1, ddof=1, keepdims=True), n)
            st["num_update_y"] = n + 1
            return x
        if self.learn_x:
            n = float(st.get("num_update_x", 0.0))
            update("mean_x", x.mean(-1, keepdims=True), n)
            update("std_x", x.std(-1, ddof=1, keepdims=True), n)
            st["num_update_x"] = n + 1
        if float(st.get("num_update_x", 1.0)) and float(st.get("num_update_y", 1.0)):
            x = (x - st["mean_x"][:bs]) / (st["std_x"][:bs] + 1e-5)
            x = x * st["std_y"][:bs] + st["mean_y"][:bs]
        return x

    @staticmethod
    def fresh_adain_state(modules, max_batch: int = 64):
        """Reference-initialised buffers (rave/blocks.py:858-868) for (name, C) pairs."""
        return {n: {"mean_x": np.zeros((max_batch, c, 1)), "std_x": np.ones((max_batch, c, 1)),
                    "mean_y": np.zeros((max_batch, c, 1)), "std_y": np.ones((max_batch, c, 1)),
                    "num_update_x": 0.0, "num_update_y": 0.0} for n, c in modules}

    def _dilated_residual(self, x, res, d):
        unit = f"{res}.aligned.branches.0.net"
        h = self._act(x, f"{unit}.0")
        h = self._conv(h, f"{unit}.1", self.cfg.kernel_size, dilation=d)
        h = self._act(h, f"{unit}.2")
        h = self._conv(h, f"{unit}.3", 1)
        return x + h

    # -------------------------------------------------------------- pqmf
    def pqmf_analysis(self, x: np.ndarray) -> np.ndarray:
        """CachedPQMF.forward: conv(1->16, k=513, stride 16) + reverse_half."""
        k = self.hkf.shape[-1]
        y = conv1d(x, self.hkf, None, stride=self.hk.shape[0], pad=get_padding(k, causal=self.cfg.causal))
        return reverse_half(y)

    def pqmf_synthesis(self, x: np.ndarray) -> np.ndarray:
        """CachedPQMF.inverse: reverse_half -> conv(16->16, k=33)*16 -> flip ->
        interleave out[m*n + j] = y[m-1-j][n]."""
        m = self.hk.shape[0]
        x = reverse_half(np.asarray(x, F64))
        k = self.hki.shape[-1]
        y = conv1d(x, self.hki, None, pad=get_padding(k, causal=self.cfg.causal)) * m
        y = y[:, ::-1, :]
        B, _, T = y.shape
        return y.transpose(0, 2, 1).reshape(B, 1, T * m)

    # -------------------------------------------------------------- encoder
    def encoder(self, x: np.ndarray) -> np.ndarray:
        """EncoderV2.forward (rave/blocks.py:508-597)."""
        cfg = self.cfg
        pre = "encoder.encoder.net"
        i = 0
        x = self._conv(x, f"{pre}.{i}", 2 * cfg.kernel_size + 1)
        i += 1
        for r, dils in zip(cfg.ratios, cfg.dilations):
            for d in dils:
                if cfg.adain:
                    x = self._adain(x, f"{pre}.{i}")
                    i += 1
                x = self._dilated_residual(x, f"{pre}.{i}", d)
                i += 1
            x = self._act(x, f"{pre}.{i}")
            i += 1
            x = self._conv(x, f"{pre}.{i}", 2 * r, stride=r)
            i += 1
        x = self._act(x, f"{pre}.{i}")
        i += 1
        return self._conv(x, f"{pre}.{i}", cfg.kernel_size)

    def encode(self, x: np.ndarray) -> np.ndarray:
        """RAVE.encode (rave/model.py:594-622)."""
        bands = self.pqmf_analysis(x)
        z = self.encoder(bands[:, :self.cfg.enc_bands])
        if self.cfg.rvq is not None:
            return z
        return self.cat_speaker(z)

    def cat_speaker(self, z):
        emb = np.broadcast_to(self.speaker.reshape(1, -1, 1), (z.shape[0], self.speaker.size, z.shape[-1]))
        return np.concatenate([z, emb], 1)

    # -------------------------------------------------------------- decoder
    def decoder_features(self, z: np.ndarray) -> np.ndarray:
        cfg = self.cfg
        pre = "decoder.net"
        i = 0
        x = self._conv(z, f"{pre}.{i}", cfg.kernel_size)
        i += 1
        for r, dils in zip(cfg.ratios[::-1], cfg.dilations[::-1]):
            x = self._act(x, f"{pre}.{i}")
            i += 1
            name = f"{pre}.{i}"
            w = fold_wn(self.p[name + ".weight_g"], self.p[name + ".weight_v"])
            x = conv_transpose1d(x, w, r, r // 2, self._b(name))
            if self.record:
                self.trace[name] = x
            i += 1
            for d in dils:
                if cfg.adain:
                    x = self._adain(x, f"{pre}.{i}")
                    i += 1
                x = self._dilated_residual(x, f"{pre}.{i}", d)
                i += 1
        x = self._act(x, f"{pre}.{i}")
        i += 1
        return x, i

    def decoder(self, z: np.ndarray, noise_u: Optional[np.ndarray] = None) -> np.ndarray:
        """GeneratorV2.forward (rave/blocks.py:692-707)."""
        cfg = self.cfg
        x, i = self.decoder_features(z)
        noise = 0.0
        wave = "decoder.waveform_module" if cfg.noise is not None else f"decoder.net.{i}"
        if cfg.noise is not None:
            if noise_u is None:
                raise ValueError("noise synthesizer needs the uniform noise tensor")
            noise = self.noise_generator(x, noise_u)
        y = self._conv(x, wave, 2 * cfg.kernel_size + 1)
        if cfg.amplitude_modulation:
            a, amp = np.split(y, 2, axis=1)
            y = a * (1.0 / (1.0 + np.exp(-amp)))
        return np.tanh(y + noise)

    def noise_generator(self, x, noise_u):
        """NoiseGeneratorV2.forward (rave/blocks.py:281-291)."""
        nz = self.cfg.noise
        pre = "decoder.noise_module.net"
        j = 0
        for i, r in enumerate(nz.ratios):
            if i > 0:
                x = self._act(x, f"{pre}.{j - 1}")
            x = self._conv(x, f"{pre}.{j}", 2 * r, stride=r, wn=False, pad=(r, 0))
            j += 2
        amp = 2 * (1.0 / (1.0 + np.exp(-(x - 5)))) ** 2.3 + 1e-7       # mod_sigmoid(x - 5)
        amp = amp.transpose(0, 2, 1)
        B, F, _ = amp.shape
        amp = amp.reshape(B, F, self.cfg.n_band, -1)
        target = int(np.prod(nz.ratios))
        ir = np.fft.irfft(amp.astype(complex), axis=-1)               # amp_to_impulse_response
        fs = ir.shape[-1]
        ir = np.roll(ir, fs // 2, -1)
        win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(fs) / fs)     # torch.hann_window (periodic)
        ir = ir * win
        ir = np.pad(ir, [(0, 0)] * 3 + [(0, target - fs)])
        ir = np.roll(ir, -fs // 2, -1)
        noise = np.asarray(noise_u, F64) * 2 - 1
        sig = np.pad(noise, [(0, 0)] * 3 + [(0, noise.shape[-1])])  # fft_convolve
        ker = np.pad(ir, [(0, 0)] * 3 + [(ir.shape[-1], 0)])
        out = np.fft.irfft(np.fft.rfft(sig) * np.fft.rfft(ker), n=sig.shape[-1])
        out = out[..., out.shape[-1] // 2:]
        out = out.transpose(0, 2, 1, 3)
        return out.reshape(out.shape[0], out.shape[1], -1)

    def decode(self, z: np.ndarray, noise_u: Optional[np.ndarray] = None) -> np.ndarray:
        """RAVE.decode (rave/model.py:624-629)."""
        return self.pqmf_synthesis(self.decoder(z, noise_u))

    def forward(self, x: np.ndarray, noise_u: Optional[np.ndarray] = None) -> np.ndarray:
        z = self.encode(x)
        if self.cfg.rvq is not None:
            z = self.cat_speaker(self.rvq_decode(self.rvq_encode(z)))
        return self.decode(z, noise_u)

    # -------------------------------------------------------------- RVQ
    def codebooks(self):
        return [np.asarray(self.p[f"encoder.rvq.layers.{i}._codebook.embed"], F64)
                for i in range(self.cfg.rvq.num_quantizers)]

    def rvq_encode(self, z: np.ndarray, return_gaps: bool = False):
        """ResidualVectorQuantization.encode (rave/quantization.py:302-311)."""
        res = np.asarray(z, F64)
        B, D, T = res.shape
        idx, gaps = [], []
        for E in self.codebooks():
            x = res.transpose(0, 2, 1).reshape(-1, D)
            dist = -((x ** 2).sum(1, keepdims=True) - 2 * x @ E.T + (E ** 2).sum(1)[None])
            ind = dist.argmax(-1)
            srt = np.sort(dist, -1)
            gaps.append(srt[:, -1] - srt[:, -2])
            q = E[ind].reshape(B, T, D).transpose(0, 2, 1)
            res = res - q
            idx.append(ind.reshape(B, T))
        out = np.stack(idx, 1)
        return (out, np.stack(gaps, 0)) if return_gaps else out

    def rvq_decode(self, idx: np.ndarray) -> np.ndarray:
        """ResidualVectorQuantization.decode (rave/quantization.py:313-318)."""
        out = 0.0
        for i, E in enumerate(self.codebooks()):
            out = out + E[idx[:, i]].transpose(0, 2, 1)
        return out
