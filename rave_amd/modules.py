"""The reference's module tree written against the ``cc`` operator seam.

rave/blocks.py builds EncoderV2 (:508-597), GeneratorV2 (:600-710),
Residual (:32-46), DilatedUnit (:84-113), NoiseGeneratorV2 (:244-291) and
AdaptiveInstanceNormalization (:856-919) out of ``cc.Conv1d`` /
``cc.ConvTranspose1d`` / ``cc.CachedSequential`` / ``cc.AlignBranches``.  The
classes below restate that construction over ``rave_amd.cc`` (whose operators
run the HIP kernels), with the same child order -- so the reference's
state_dict names (``encoder.encoder.net.1.aligned.branches.0.net.1.weight``,
``decoder.net.2.weight``, ``decoder.noise_module.net.0.weight``,
``encoder.encoder.net.1.mean_x``, ...) load unchanged -- and the same
cached-mode delay bookkeeping when ``cc.use_cached_conv(True)`` is set before
construction.  ``RAVEModules`` is RAVE.encode / decode / forward
(rave/model.py:594-634): PQMF, the first ``enc_bands`` bands, the encoder, the
speaker concat; the decoder, the PQMF inverse.  Every config of the path is
covered: v2 / causal / discrete (the encoder output; RVQ through
``cc.rvq_encode`` / ``rvq_decode``), Snake, AdaIN and the noise synthesizer.

No stock PyTorch kernel runs on the path: every activation module is fused
into the prologue of the convolution after it (each keeps its own parameters,
e.g. Snake's ``alpha``, and reports them through ``fused()``), each Residual's
sum rides in its last conv's epilogue (``residual=``), the delay lines run on
rave_copy (``cc.CachedPadding1d``), AdaIN and the noise filter stage on their
own kernels, and GeneratorV2's epilogue (amplitude modulation, noise, tanh)
inside the PQMF synthesis (``RAVEModules.decode``).  Calling an activation or
GeneratorV2 on its own still works (torch elementwise ops): that is the
standalone module, not the path.  Everything is TorchScript-scriptable.

This is the operator-level drop-in; the fused, autotuned engine
(rave_amd.RAVE) is the fast path.
"""
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import cc

ACT_NONE, ACT_LEAKY, ACT_SNAKE = cc.ACT_NONE, cc.ACT_LEAKY, cc.ACT_SNAKE


class Snake(nn.Module):
    """rave/blocks.py:845-853: x + (alpha + 1e-9)^-1 sin(alpha x)^2 (the conv
    after it applies it, from ``fused()``)."""

    def __init__(self, dim: int):
        super().__init__()
        self.alpha = nn.Parameter(torch.ones(dim, 1))

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, act: int = -1, slope: float = 0.2,
                alpha: Optional[torch.Tensor] = None) -> torch.Tensor:
        return x + (self.alpha + 1e-9).reciprocal() * (self.alpha * x).sin().pow(2)

    @torch.jit.export
    def fused(self) -> Tuple[int, float, Optional[torch.Tensor]]:
        return 2, 0.0, self.alpha.reshape(-1)          # ACT_SNAKE


class LeakyReLU(nn.Module):
    """nn.LeakyReLU(.2) (rave/blocks.py:91, the default activation)."""

    def __init__(self, negative_slope: float = 0.2):
        super().__init__()
        self.negative_slope = float(negative_slope)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, act: int = -1, slope: float = 0.2,
                alpha: Optional[torch.Tensor] = None) -> torch.Tensor:
        return torch.nn.functional.leaky_relu(x, self.negative_slope)

    @torch.jit.export
    def fused(self) -> Tuple[int, float, Optional[torch.Tensor]]:
        return 1, self.negative_slope, None            # ACT_LEAKY


def _activation(kind: str, dim: int) -> nn.Module:
    return Snake(dim) if kind == "snake" else LeakyReLU(0.2)


class FusedSequential(cc.CachedSequential):
    """cc.CachedSequential whose activation children are fused into the conv
    that follows them: an activation's ``fused()`` (kind, slope, alpha) is
    handed to the next child's call, which applies it in its prologue.  Every
    child takes ``(x, residual, act, slope, alpha)`` and reports ``fused()``
    (non-activations report ACT_NONE)."""

    def run(self, x: torch.Tensor, act: int, slope: float,
            alpha: Optional[torch.Tensor]) -> Tuple[torch.Tensor, int, float, Optional[torch.Tensor]]:
        """Run the children; returns the output and a trailing activation not yet applied."""
        for m in self:
            a, s, al = m.fused()
            if a != 0:                  # an activation: applied by the next child
                act, slope, alpha = a, s, al
            else:
                x = m(x, None, act if act != 0 else -1, slope, alpha)
                act, slope, alpha = 0, 0.0, None
        return x, act, slope, alpha

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y, act, _, _ = self.run(x, 0, 0.0, None)
        if act != 0:
            raise RuntimeError("FusedSequential: an activation must be followed by a convolution")
        return y


class Residual(nn.Module):
    """AlignBranches(module, Identity, delays=[module delay, 0]); the sum is
    the module's last conv's epilogue (rave/blocks.py:32-46)."""

    def __init__(self, module: nn.Module, cumulative_delay: int = 0):
        super().__init__()
        d = int(module.cumulative_delay)
        self.aligned = cc.AlignBranches(module, nn.Identity(), delays=[d, 0])
        self.cumulative_delay = d + cumulative_delay

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, act: int = -1, slope: float = 0.2,
                alpha: Optional[torch.Tensor] = None) -> torch.Tensor:
        assert act <= 0 and residual is None
        x_net = self.aligned.paddings[0](x)
        x_res = self.aligned.paddings[1](x)
        return self.aligned.branches[0](x_net, x_res)

    @torch.jit.export
    def fused(self) -> Tuple[int, float, Optional[torch.Tensor]]:
        return 0, 0.0, None                            # ACT_NONE


class DilatedUnit(nn.Module):
    """act -> Conv1d(k, dilation d) -> act -> Conv1d(1) (rave/blocks.py:84-113);
    each activation in its conv's prologue, ``residual`` added by the last conv."""

    def __init__(self, dim: int, kernel_size: int, dilation: int, activation: str = "leaky"):
        super().__init__()
        self.net = cc.CachedSequential(
            _activation(activation, dim),
            cc.Conv1d(dim, dim, kernel_size, dilation=dilation, padding=cc.get_padding(kernel_size, dilation=dilation)),
            _activation(activation, dim),
            cc.Conv1d(dim, dim, 1))
        self.cumulative_delay = int(self.net[1].cumulative_delay)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        a0, s0, al0 = self.net[0].fused()
        h = self.net[1](x, None, a0, s0, al0)
        a2, s2, al2 = self.net[2].fused()
        return self.net[3](h, residual, a2, s2, al2)


class AdaptiveInstanceNormalization(nn.Module):
    """rave/blocks.py:856-919, eval mode, on the rave_adain kernel: the
    reference's buffers (per-row statistics of MAX_BATCH_SIZE rows, learn
    flags, update counters), transfer / learn_x / learn_y."""

    def __init__(self, dim: int):
        super().__init__()
        mb = cc.MAX_BATCH_SIZE
        self.register_buffer("mean_x", torch.zeros(mb, dim, 1))
        self.register_buffer("std_x", torch.ones(mb, dim, 1))
        self.register_buffer("learn_x", torch.zeros(1))
        self.register_buffer("num_update_x", torch.zeros(1))
        self.register_buffer("mean_y", torch.zeros(mb, dim, 1))
        self.register_buffer("std_y", torch.ones(mb, dim, 1))
        self.register_buffer("learn_y", torch.zeros(1))
        self.register_buffer("num_update_y", torch.zeros(1))

    @torch.jit.export
    def reset_x(self) -> None:
        self.mean_x.zero_()
        self.std_x.fill_(1.0)
        self.num_update_x.zero_()

    @torch.jit.export
    def reset_y(self) -> None:
        self.mean_y.zero_()
        self.std_y.fill_(1.0)
        self.num_update_y.zero_()

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, act: int = -1, slope: float = 0.2,
                alpha: Optional[torch.Tensor] = None) -> torch.Tensor:
        assert act <= 0 and residual is None
        if self.training:
            return x
        mode = 0
        if bool(self.learn_y):
            mode = 2
        elif bool(self.learn_x):
            mode = 1
        return cc.adain(x, self.mean_x, self.std_x, self.mean_y, self.std_y, self.num_update_x, self.num_update_y,
                        mode)

    @torch.jit.export
    def fused(self) -> Tuple[int, float, Optional[torch.Tensor]]:
        return 0, 0.0, None                            # ACT_NONE


class EncoderV2(nn.Module):
    """conv k(2ks+1) -> [(AdaIN,) Residual(DilatedUnit) per dilation, act, strided
    conv k 2r] per ratio -> act -> conv ks (rave/blocks.py:508-597; no
    spectrogram, no GRU in v2)."""

    def __init__(self, data_size: int, capacity: int, ratios, latent_size: int, n_out: int, kernel_size: int,
                 dilations, activation: str = "leaky", adain: bool = False):
        super().__init__()
        if isinstance(dilations[0], int):
            dilations = [dilations for _ in ratios]
        net: List[nn.Module] = [cc.Conv1d(data_size, capacity, kernel_size * 2 + 1,
                                          padding=cc.get_padding(kernel_size * 2 + 1))]
        ch = capacity
        for r, dils in zip(ratios, dilations):
            for d in dils:
                if adain:
                    net.append(AdaptiveInstanceNormalization(ch))
                net.append(Residual(DilatedUnit(ch, kernel_size, d, activation)))
            net.append(_activation(activation, ch))
            net.append(cc.Conv1d(ch, 2 * ch, 2 * r, stride=r, padding=cc.get_padding(2 * r, r)))
            ch *= 2
        net.append(_activation(activation, ch))
        net.append(cc.Conv1d(ch, latent_size * n_out, kernel_size, padding=cc.get_padding(kernel_size)))
        self.net = FusedSequential(*net)

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


class NoiseGeneratorV2(nn.Module):
    """rave/blocks.py:244-291: strided convs (k 2r, padding (r, 0), activation
    between them) -> pre-sigmoid band amplitudes -> the filter stage
    (mod_sigmoid, amp_to_impulse_response, fft_convolve against U[0,1) noise:
    rave/core.py:66-129) on the rave_noise_synth kernel."""

    def __init__(self, in_size: int, hidden_size: int, data_size: int, ratios, noise_bands: int,
                 activation: str = "leaky"):
        super().__init__()
        channels = [in_size] + (len(ratios) - 1) * [hidden_size] + [data_size * noise_bands]
        net: List[nn.Module] = []
        for i, r in enumerate(ratios):
            net.append(cc.Conv1d(channels[i], channels[i + 1], 2 * r, padding=(r, 0), stride=r))
            if i != len(ratios) - 1:
                net.append(_activation(activation, channels[i + 1]))
        self.net = FusedSequential(*net)
        self.data_size = int(data_size)
        self.noise_bands = int(noise_bands)
        target = 1
        for r in ratios:
            target *= int(r)
        self.target = target
        self.register_buffer("target_size", torch.tensor(target).long())

    def forward(self, x: torch.Tensor, noise_u: Optional[torch.Tensor] = None, act: int = ACT_NONE,
                slope: float = 0.2, alpha: Optional[torch.Tensor] = None) -> torch.Tensor:
        """x: the decoder features (``act``: their activation, not yet applied);
        ``noise_u``: the U[0,1) draw (B, F, data_size, target), or None (drawn
        here, as the reference's torch.rand_like)."""
        amp, _, _, _ = self.net.run(x, act, slope, alpha)
        if noise_u is None:
            noise_u = torch.rand(amp.shape[0], amp.shape[-1], self.data_size, self.target, device=amp.device)
        return cc.noise_synth(amp, noise_u, self.data_size, self.noise_bands)


class GeneratorV2(nn.Module):
    """conv ks (latent -> 2^len(ratios) capacity) -> [act, ConvTranspose(2r, r, r//2),
    (AdaIN,) Residual(DilatedUnit) per dilation] per reversed ratio -> act ->
    conv k(2ks+1) (the waveform module), with the noise module beside it ->
    x * sigmoid(a) + noise -> tanh (rave/blocks.py:600-710)."""

    def __init__(self, data_size: int, capacity: int, ratios, latent_size: int, kernel_size: int, dilations,
                 amplitude_modulation: bool = True, activation: str = "leaky", adain: bool = False,
                 noise=None):
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
                if adain:
                    net.append(AdaptiveInstanceNormalization(ch))
                net.append(Residual(DilatedUnit(ch, kernel_size, d, activation)))
        net.append(_activation(activation, ch))
        waveform = cc.Conv1d(ch, data_size * 2 if amplitude_modulation else data_size, kernel_size * 2 + 1,
                             padding=cc.get_padding(kernel_size * 2 + 1))
        if noise is not None:
            self.waveform_module = waveform
            self.noise_module = NoiseGeneratorV2(ch, noise.hidden_size, data_size, list(noise.ratios),
                                                 noise.noise_bands, activation)
        else:
            net.append(waveform)
            self.waveform_module = None
            self.noise_module = None
        self.net = FusedSequential(*net)
        self.amplitude_modulation = bool(amplitude_modulation)

    @torch.jit.export
    def features(self, x: torch.Tensor, noise_u: Optional[torch.Tensor] = None
                 ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
        """Everything before the epilogue: the waveform conv's output and the
        noise (None without a noise module)."""
        h, act, slope, alpha = self.net.run(x, 0, 0.0, None)
        noise: Optional[torch.Tensor] = None
        if self.noise_module is not None:
            # the trailing activation feeds both the noise module's first conv and the waveform conv
            noise = self.noise_module(h, noise_u, act, slope, alpha)
            h = self.waveform_module(h, None, act, slope, alpha)
        return h, noise

    def forward(self, x: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The standalone module (its epilogue as torch elementwise ops; RAVEModules.decode
        fuses it into the PQMF synthesis instead)."""
        h, noise = self.features(x, noise_u)
        if self.amplitude_modulation:
            n = h.shape[1] // 2
            h = h[:, :n] * torch.sigmoid(h[:, n:])
        if noise is not None:
            h = h + noise
        return torch.tanh(h)


class RAVEModules(nn.Module):
    """RAVE.encode / decode / forward (rave/model.py:594-634) over the module tree."""

    def __init__(self, cfg, speaker=None, hk=None):
        super().__init__()
        import numpy as np
        cc.set_padding_mode("causal" if cfg.causal else "centered")
        try:
            self.pqmf = cc.CachedPQMF(cfg.pqmf_attenuation, cfg.n_band, hk=hk)
            enc = EncoderV2(cfg.enc_bands, cfg.capacity, cfg.ratios, cfg.latent_size, 1, cfg.kernel_size,
                            [list(d) for d in cfg.dilations], cfg.activation, cfg.adain)
            self.encoder = VariationalEncoder(enc)
            self.decoder = GeneratorV2(cfg.n_band, cfg.capacity, cfg.ratios, cfg.dec_in, cfg.kernel_size,
                                       [list(d) for d in cfg.dilations], cfg.amplitude_modulation, cfg.activation,
                                       cfg.adain, cfg.noise)
        finally:
            cc.set_padding_mode("centered")
        spk = np.zeros(cfg.speaker_size, np.float32) if speaker is None else np.asarray(speaker, np.float32)
        self.register_buffer("speaker", torch.from_numpy(spk.reshape(-1)))
        self.enc_bands = int(cfg.enc_bands)
        self.discrete = cfg.rvq is not None
        self.epilogue = 1 if cfg.amplitude_modulation else 2      # pqmf_synthesis mode

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        z = self.encoder(self.pqmf(x, self.enc_bands))
        if self.discrete:
            return z
        emb = self.speaker.reshape(1, -1, 1).expand(z.shape[0], -1, z.shape[-1])
        return torch.cat([z, emb], 1)

    def decode(self, z: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        """GeneratorV2 then CachedPQMF.inverse, the generator's epilogue
        (AM, noise, tanh) fused into the synthesis."""
        h, noise = self.decoder.features(z, noise_u)
        return self.pqmf.inverse(h, self.epilogue, noise)

    def forward(self, x: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.decode(self.encode(x), noise_u)


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
    buffers = {n for n, _ in m.named_buffers()}
    missing = [k for k in own if k not in sd and k not in ("speaker", "pqmf.hk") and k not in buffers]
    if missing:
        raise KeyError(f"parameters not in the dict: {missing[:5]}")
