"""The reference's module tree written against the ``cc`` operator seam.

rave/blocks.py builds EncoderV2 (:508-597), GeneratorV2 (:600-710),
Residual (:32-46) and DilatedUnit (:84-113) out of ``cc.Conv1d`` /
``cc.ConvTranspose1d`` / ``cc.CachedSequential`` / ``cc.AlignBranches``.  The
classes below restate that construction over ``rave_amd.cc`` (whose operators
run the HIP kernels), with the same child order -- so the reference's
state_dict names (``encoder.encoder.net.1.aligned.branches.0.net.1.weight``,
``decoder.net.2.weight``, ...) load unchanged -- and the same cached-mode
delay bookkeeping when ``cc.use_cached_conv(True)`` is set before
construction.  ``RAVEModules`` is RAVE.encode / decode / forward
(rave/model.py:594-634): PQMF, the first ``enc_bands`` bands, the encoder, the
speaker concat; the decoder, the PQMF inverse.  v2 / causal / discrete (the
encoder output; RVQ through ``cc.rvq_encode`` / ``rvq_decode``) and the
Snake activation are covered; AdaIN and the noise synthesizer run on the
engine (rave_amd.RAVE).  Everything is TorchScript-scriptable.

This is the operator-level drop-in; the fused, autotuned engine
(rave_amd.RAVE) is the fast path.
"""
from typing import List

import torch
import torch.nn as nn

from . import cc


class Snake(nn.Module):
    """rave/blocks.py:845-853: x + (alpha + 1e-9)^-1 sin(alpha x)^2."""

    def __init__(self, dim: int):
        super().__init__()
        self.alpha = nn.Parameter(torch.ones(dim, 1))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return x + (self.alpha + 1e-9).reciprocal() * (self.alpha * x).sin().pow(2)


def _activation(kind: str, dim: int) -> nn.Module:
    return Snake(dim) if kind == "snake" else nn.LeakyReLU(0.2)


class Residual(nn.Module):
    """AlignBranches(module, Identity, delays=[module delay, 0]); the sum."""

    def __init__(self, module: nn.Module, cumulative_delay: int = 0):
        super().__init__()
        d = int(module.cumulative_delay)
        self.aligned = cc.AlignBranches(module, nn.Identity(), delays=[d, 0])
        self.cumulative_delay = d + cumulative_delay

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y: List[torch.Tensor] = self.aligned(x)
        return y[0] + y[1]


class DilatedUnit(nn.Module):
    """act -> Conv1d(k, dilation d) -> act -> Conv1d(1)."""

    def __init__(self, dim: int, kernel_size: int, dilation: int, activation: str = "leaky"):
        super().__init__()
        self.net = cc.CachedSequential(
            _activation(activation, dim),
            cc.Conv1d(dim, dim, kernel_size, dilation=dilation, padding=cc.get_padding(kernel_size, dilation=dilation)),
            _activation(activation, dim),
            cc.Conv1d(dim, dim, 1))
        self.cumulative_delay = int(self.net[1].cumulative_delay)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.net(x)


class EncoderV2(nn.Module):
    """conv k(2ks+1) -> [Residual(DilatedUnit) per dilation, act, strided conv k 2r] per
    ratio -> act -> conv ks (rave/blocks.py:508-597; no spectrogram, no GRU in v2)."""

    def __init__(self, data_size: int, capacity: int, ratios, latent_size: int, n_out: int, kernel_size: int,
                 dilations, activation: str = "leaky"):
        super().__init__()
        if isinstance(dilations[0], int):
            dilations = [dilations for _ in ratios]
        net: List[nn.Module] = [cc.Conv1d(data_size, capacity, kernel_size * 2 + 1,
                                          padding=cc.get_padding(kernel_size * 2 + 1))]
        ch = capacity
        for r, dils in zip(ratios, dilations):
            for d in dils:
                net.append(Residual(DilatedUnit(ch, kernel_size, d, activation)))
            net.append(_activation(activation, ch))
            net.append(cc.Conv1d(ch, 2 * ch, 2 * r, stride=r, padding=cc.get_padding(2 * r, r)))
            ch *= 2
        net.append(_activation(activation, ch))
        net.append(cc.Conv1d(ch, latent_size * n_out, kernel_size, padding=cc.get_padding(kernel_size)))
        self.net = cc.CachedSequential(*net)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.net(x)


class VariationalEncoder(nn.Module):
    """The wrapper whose ``encoder`` child gives the ``encoder.encoder.*`` names;
    RAVE.encode does not reparametrize (rave/model.py:621)."""

    def __init__(self, encoder: nn.Module):
        super().__init__()
        self.encoder = encoder

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.encoder(x)


class GeneratorV2(nn.Module):
    """conv ks (latent -> 2^len(ratios) capacity) -> [act, ConvTranspose(2r, r, r//2),
    Residual(DilatedUnit) per dilation] per reversed ratio -> act -> conv
    k(2ks+1) -> x * sigmoid(a) -> tanh (rave/blocks.py:600-710, no noise)."""

    def __init__(self, data_size: int, capacity: int, ratios, latent_size: int, kernel_size: int, dilations,
                 amplitude_modulation: bool = True, activation: str = "leaky"):
        super().__init__()
        if isinstance(dilations[0], int):
            dilations = [dilations for _ in ratios]
        dilations = list(dilations)[::-1]
        ratios = list(ratios)[::-1]
        ch = (2 ** len(ratios)) * capacity
        net: List[nn.Module] = [cc.Conv1d(latent_size, ch, kernel_size, padding=cc.get_padding(kernel_size))]
        for r, dils in zip(ratios, dilations):
            net.append(_activation(activation, ch))
            net.append(cc.ConvTranspose1d(ch, ch // 2, 2 * r, stride=r, padding=r // 2))
            ch //= 2
            for d in dils:
                net.append(Residual(DilatedUnit(ch, kernel_size, d, activation)))
        net.append(_activation(activation, ch))
        net.append(cc.Conv1d(ch, data_size * 2 if amplitude_modulation else data_size, kernel_size * 2 + 1,
                             padding=cc.get_padding(kernel_size * 2 + 1)))
        self.net = cc.CachedSequential(*net)
        self.amplitude_modulation = bool(amplitude_modulation)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.net(x)
        if self.amplitude_modulation:
            n = x.shape[1] // 2
            x = x[:, :n] * torch.sigmoid(x[:, n:])
        return torch.tanh(x)


class RAVEModules(nn.Module):
    """RAVE.encode / decode / forward (rave/model.py:594-634) over the module tree."""

    def __init__(self, cfg, speaker=None, hk=None):
        super().__init__()
        import numpy as np
        if cfg.noise is not None or cfg.adain:
            raise NotImplementedError("AdaIN / NoiseGeneratorV2 configs run on the engine (rave_amd.RAVE)")
        cc.set_padding_mode("causal" if cfg.causal else "centered")
        self.pqmf = cc.CachedPQMF(cfg.pqmf_attenuation, cfg.n_band, hk=hk)
        enc = EncoderV2(cfg.enc_bands, cfg.capacity, cfg.ratios, cfg.latent_size, 1, cfg.kernel_size,
                        [list(d) for d in cfg.dilations], cfg.activation)
        self.encoder = VariationalEncoder(enc)
        self.decoder = GeneratorV2(cfg.n_band, cfg.capacity, cfg.ratios, cfg.dec_in, cfg.kernel_size,
                                   [list(d) for d in cfg.dilations], cfg.amplitude_modulation, cfg.activation)
        spk = np.zeros(cfg.speaker_size, np.float32) if speaker is None else np.asarray(speaker, np.float32)
        self.register_buffer("speaker", torch.from_numpy(spk.reshape(-1)))
        self.enc_bands = int(cfg.enc_bands)
        self.discrete = cfg.rvq is not None
        cc.set_padding_mode("centered")

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        z = self.encoder(self.pqmf(x, self.enc_bands))
        if self.discrete:
            return z
        emb = self.speaker.reshape(1, -1, 1).expand(z.shape[0], -1, z.shape[-1])
        return torch.cat([z, emb], 1)

    def decode(self, z: torch.Tensor) -> torch.Tensor:
        return self.pqmf.inverse(self.decoder(z))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.decode(self.encode(x))


def load_reference_state(m: nn.Module, params) -> None:
    """Load a reference-named parameter dict (``weight_g`` / ``weight_v`` folded,
    as scripts/export.py:598-600 removes weight norm) into a module tree."""
    import numpy as np
    from .weights import fold_weight_norm
    sd = {}
    for k, v in params.items():
        if k.endswith(".weight_g"):
            base = k[:-len(".weight_g")]
            sd[base + ".weight"] = torch.from_numpy(fold_weight_norm(np.asarray(v), np.asarray(params[base + ".weight_v"])))
        elif not k.endswith(".weight_v"):
            sd[k] = torch.from_numpy(np.array(v, np.float32))
    own = m.state_dict()
    for k, v in sd.items():
        if k in own:
            own[k].copy_(v.reshape(own[k].shape))
        elif not k.startswith("encoder.rvq."):
            raise KeyError(f"{k}: not in the module tree")
    missing = [k for k in own if k not in sd and k not in ("speaker", "pqmf.hk")]
    if missing:
        raise KeyError(f"parameters not in the dict: {missing[:5]}")
