"""Model hyper-parameters for the RAVE encode->decode path.

Each preset restates the gin bindings of one reference config file; the gin
files are the source of truth for shapes:

* ``v2``       -- rave/configs/v1.gin:13-41 + rave/configs/v2.gin:15-60
* ``causal``   -- v2 + rave/configs/causal.gin:5 (``cc.get_padding.mode = 'causal'``)
* ``discrete`` -- rave/configs/discrete.gin:14-40 (CAPACITY 96, LATENT 128, 16x1024 RVQ)
* ``v3``       -- rave/configs/v3.gin:3-6 (v2 + adain.gin + snake.gin)
* ``v3_noise`` -- v3 + rave/configs/noise.gin:5-11 (NoiseGeneratorV2)

Fork-specific facts: the encoder reads only the first
``data_size = 6`` PQMF bands (rave/model.py:613) and ``encode`` appends a
constant 256-d speaker embedding (rave/model.py:618-620), so the decoder's input
width is ``latent + 256`` (rave/core.py:78-79).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import List, Optional, Tuple


@dataclass(frozen=True)
class NoiseConfig:
    """rave/configs/noise.gin:8-11 / NoiseGeneratorV2 (rave/blocks.py:247-279)."""
    hidden_size: int = 128
    ratios: Tuple[int, ...] = (2, 2, 2)
    noise_bands: int = 5


@dataclass(frozen=True)
class RVQConfig:
    """rave/configs/discrete.gin:14-17,37-40 / ResidualVectorQuantization."""
    num_quantizers: int = 16
    codebook_size: int = 1024


@dataclass(frozen=True)
class RaveConfig:
    name: str = "v2"
    n_band: int = 16                       # v1.gin:15
    pqmf_attenuation: float = 100.0        # v1.gin:38
    enc_bands: int = 6                     # v2.gin:40 data_size = 6, model.py:613
    capacity: int = 64                     # v2.gin:22
    ratios: Tuple[int, ...] = (4, 4, 2, 2)  # v2.gin:21
    latent_size: int = 64                  # v1.gin:16
    kernel_size: int = 3                   # v2.gin:15
    dilations: Tuple[Tuple[int, ...], ...] = ((1, 3, 9), (1, 3, 9), (1, 3, 9), (1, 3))
    speaker_size: int = 256                # v2.gin:25
    amplitude_modulation: bool = True      # v2.gin:59
    causal: bool = False                   # causal.gin:5
    activation: str = "leaky"              # LeakyReLU(.2) default; 'snake' per snake.gin
    leaky_slope: float = 0.2               # rave/blocks.py:91
    adain: bool = False                    # adain.gin
    noise: Optional[NoiseConfig] = None    # noise.gin
    rvq: Optional[RVQConfig] = None        # discrete.gin
    conv_bias: bool = True                 # v1.gin:33 cc.Conv1d.bias = True
    convt_bias: bool = False               # v1.gin:34 cc.ConvTranspose1d.bias = False

    # ------------------------------------------------------------------ derived
    @property
    def hop(self) -> int:
        """Audio samples per latent frame: n_band * prod(ratios) (= 1024 for v2)."""
        h = self.n_band
        for r in self.ratios:
            h *= r
        return h

    @property
    def dec_in(self) -> int:
        """Decoder input channels: latent + speaker (rave/core.py:78-79)."""
        return self.latent_size + self.speaker_size

    @property
    def dec_out(self) -> int:
        """Waveform conv output channels (rave/blocks.py:671-677)."""
        return self.n_band * 2 if self.amplitude_modulation else self.n_band

    @property
    def dec_channels(self) -> int:
        """First decoder width 2**len(ratios) * capacity (rave/blocks.py:617-620)."""
        return (2 ** len(self.ratios)) * self.capacity

    def replace(self, **kw) -> "RaveConfig":
        return dataclasses.replace(self, **kw)


def v2(**kw) -> RaveConfig:
    return RaveConfig(name="v2").replace(**kw)


def causal(**kw) -> RaveConfig:
    return RaveConfig(name="causal", causal=True).replace(**kw)


def discrete(**kw) -> RaveConfig:
    return RaveConfig(name="discrete", capacity=96, latent_size=128,
                      rvq=RVQConfig()).replace(**kw)


def v3(**kw) -> RaveConfig:
    return RaveConfig(name="v3", activation="snake", adain=True).replace(**kw)


def v3_noise(**kw) -> RaveConfig:
    return RaveConfig(name="v3_noise", activation="snake", adain=True,
                      noise=NoiseConfig()).replace(**kw)


PRESETS = {"v2": v2, "causal": causal, "discrete": discrete, "v3": v3, "v3_noise": v3_noise}


def get_config(name: str, **kw) -> RaveConfig:
    if name not in PRESETS:
        raise ValueError(f"unknown config {name!r}; choose from {sorted(PRESETS)}")
    return PRESETS[name](**kw)


def get_padding(kernel_size: int, stride: int = 1, dilation: int = 1,
                causal: bool = False) -> Tuple[int, int]:
    """Restates cached_conv.get_padding (cached-conv>=2.5.0, requirements.txt:14;
    gin-bound at rave/__init__.py:25, causal.gin:5): p = (k-1)*d + 1, centered
    ((p-1)//2, p//2), causal (p-1, 0), k == 1 -> (0, 0).  ``stride`` does not
    enter the formula (the reference passes it at rave/blocks.py:571)."""
    if kernel_size == 1:
        return (0, 0)
    p = (kernel_size - 1) * dilation + 1
    if causal:
        return (p - 1, 0)
    return ((p - 1) // 2, p // 2)
