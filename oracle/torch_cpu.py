"""CPU BASELINE for bench.py -- TEST INFRASTRUCTURE ONLY.

Only tests/ and bench.py's ``cpu_baseline`` leg import this module, as the
timed CPU comparison point; the product path (rave_amd) never does.

The reference's own CPU path is torch fp32 on oneDNN: every cached_conv
operator is ``F.pad`` + ``F.conv1d`` / ``nn.ConvTranspose1d`` (rave/blocks.py,
cached-conv>=2.5.0 in non-cached mode) and everything else is elementwise torch.
The reference package itself cannot be imported on the GPU box (it is not
there, and offline it needs gin / cached_conv / lightning / a torch.hub fetch,
SURVEY.md section 8c), so this module restates the same module graph with the
same torch CPU kernels:

* CachedPQMF.forward / inverse      rave/pqmf.py:269-284 (+ reverse_half :13-17)
* EncoderV2.forward                 rave/blocks.py:508-597
* GeneratorV2.forward               rave/blocks.py:600-710 (AM + tanh :692-707)
* Residual(DilatedUnit)             rave/blocks.py:32-46, 84-113
* LeakyReLU(.2) / Snake             rave/blocks.py:91, 845-853
* RAVE.encode / decode / forward    rave/model.py:594-634

Weight norm is folded once at construction (what the reference's export does
with remove_weight_norm, scripts/export.py:598-600).  AdaIN is the eval-mode
identity; the noise synthesizer and RVQ are not restated here (bench's CPU
baseline is configs[1], v2).  Parity: tests/test_torch_cpu_baseline.py checks
it against the golden fixtures made by running the reference.
"""
from __future__ import annotations

from typing import Mapping, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .rave_oracle import fold_wn, get_padding, pqmf_filters, qmf_bank


class TorchCPURave:
    """torch fp32 CPU restatement of RAVE.encode / decode / forward."""

    def __init__(self, cfg, params: Mapping[str, np.ndarray], speaker: np.ndarray,
                 hk: Optional[np.ndarray] = None):
        if cfg.noise is not None or cfg.rvq is not None:
            raise NotImplementedError("torch CPU baseline covers the v2 / causal / v3 graphs")
        self.cfg = cfg
        hk = qmf_bank(cfg.pqmf_attenuation, cfg.n_band) if hk is None else np.asarray(hk, np.float32)
        hkf, hki = pqmf_filters(hk)
        self.m = hk.shape[0]
        self.hkf = torch.from_numpy(np.ascontiguousarray(hkf, np.float32))
        self.hki = torch.from_numpy(np.ascontiguousarray(hki, np.float32))
        self.w = {}
        for k in params:
            if k.endswith(".weight_v"):
                n = k[:-len(".weight_v")]
                self.w[n] = torch.from_numpy(fold_wn(params[n + ".weight_g"], params[k]).astype(np.float32))
            elif k.endswith(".bias") or k.endswith(".alpha"):
                self.w[k] = torch.from_numpy(np.asarray(params[k], np.float32))
        self.speaker = torch.from_numpy(np.asarray(speaker, np.float32).reshape(1, -1, 1))

    # ------------------------------------------------------------ operators
    def _act(self, x, module):
        if self.cfg.activation == "snake":
            a = self.w[module + ".alpha"].reshape(1, -1, 1)
            return x + (a + 1e-9).reciprocal() * torch.sin(a * x).pow(2)
        return F.leaky_relu(x, self.cfg.leaky_slope)

    def _conv(self, x, name, k, stride=1, dilation=1):
        x = F.pad(x, get_padding(k, stride, dilation, self.cfg.causal))
        return F.conv1d(x, self.w[name], self.w.get(name + ".bias"), stride=stride, dilation=dilation)

    def _unit(self, x, res, d):
        unit = f"{res}.aligned.branches.0.net"
        h = self._conv(self._act(x, f"{unit}.0"), f"{unit}.1", self.cfg.kernel_size, dilation=d)
        h = self._conv(self._act(h, f"{unit}.2"), f"{unit}.3", 1)
        return x + h

    @staticmethod
    def _reverse_half(x):
        mask = torch.ones_like(x)
        mask[..., 1::2, ::2] = -1
        return x * mask

    # ------------------------------------------------------------ model
    def encode(self, x: torch.Tensor) -> torch.Tensor:
        cfg = self.cfg
        k = self.hkf.shape[-1]
        bands = F.conv1d(F.pad(x, get_padding(k, causal=cfg.causal)), self.hkf, stride=self.m)
        h = self._reverse_half(bands)[:, :cfg.enc_bands]
        pre, i = "encoder.encoder.net", 0
        h = self._conv(h, f"{pre}.{i}", 2 * cfg.kernel_size + 1)
        i += 1
        for r, dils in zip(cfg.ratios, cfg.dilations):
            for d in dils:
                i += int(cfg.adain)                   # AdaIN: eval identity
                h = self._unit(h, f"{pre}.{i}", d)
                i += 1
            h = self._act(h, f"{pre}.{i}")
            i += 1
            h = self._conv(h, f"{pre}.{i}", 2 * r, stride=r)
            i += 1
        h = self._act(h, f"{pre}.{i}")
        z = self._conv(h, f"{pre}.{i + 1}", cfg.kernel_size)
        return torch.cat([z, self.speaker.expand(z.shape[0], -1, z.shape[-1])], 1)

    def decode(self, z: torch.Tensor) -> torch.Tensor:
        cfg = self.cfg
        pre, i = "decoder.net", 0
        x = self._conv(z, f"{pre}.{i}", cfg.kernel_size)
        i += 1
        for r, dils in zip(cfg.ratios[::-1], cfg.dilations[::-1]):
            x = self._act(x, f"{pre}.{i}")
            i += 1
            name = f"{pre}.{i}"
            x = F.conv_transpose1d(x, self.w[name], self.w.get(name + ".bias"), stride=r, padding=r // 2)
            i += 1
            for d in dils:
                i += int(cfg.adain)
                x = self._unit(x, f"{pre}.{i}", d)
                i += 1
        x = self._act(x, f"{pre}.{i}")
        y = self._conv(x, f"{pre}.{i + 1}", 2 * cfg.kernel_size + 1)
        if cfg.amplitude_modulation:
            a, amp = torch.split(y, y.shape[1] // 2, 1)
            y = a * torch.sigmoid(amp)
        y = torch.tanh(y)
        # CachedPQMF.inverse
        k = self.hki.shape[-1]
        y = self._reverse_half(y)
        y = F.conv1d(F.pad(y, get_padding(k, causal=cfg.causal)), self.hki) * self.m
        y = y.flip(1)
        B, _, T = y.shape
        return y.permute(0, 2, 1).reshape(B, 1, T * self.m)

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.decode(self.encode(x))
