"""TorchScript export for nn~ over the native engine.

nn~ loads a TorchScript file.  ScriptedRAVE below is scriptable: its compute
is the TORCH_LIBRARY custom class torch.classes.rave_amd.Engine
(rave_amd/csrc/torch_ops.cpp over the C-ABI engine), its nn~ surface the
reference's: register_method metadata (scripts/export.py:229-240; the
upstream encode / decode / forward table of :172-227), 1-tuple attributes
with @torch.jit.export getters / setters (:120-126, :427-479), update_adain
(:248-265), stereo decode (:317-336), and export_to_ts (:618).

Streaming (cc.use_cached_conv(True), :543) works for causal and centred
configs alike.  A discrete config exports as DiscreteScriptedRAVE
(scripts/export.py:503-517): ``encode`` returns the RVQ indices as float
(post_process_latent, ``rvq.encode(z).float()``), ``decode`` clamps them to the
codebook and truncates to int64 (pre_process_latent) before rvq.decode ->
speaker concat -> decoder.

(No ``from __future__ import annotations`` here: TorchScript must see the
attribute annotations as types.)
"""
import os as _os
from typing import List, Optional, Tuple

import torch

_TORCH_LIB = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "librave_amd_torch.so")


def load_torch_ops() -> None:
    """Register torch.classes.rave_amd.Engine (idempotent).  A host that loads
    an exported .ts (nn~) loads this library first, as for any custom op."""
    if _TORCH_LIB in torch.ops.loaded_libraries:
        return
    if not _os.path.exists(_TORCH_LIB):
        raise ImportError(f"{_TORCH_LIB} is missing (build with `make -C rave_amd/csrc`)")
    from . import _native  # noqa: F401  (loads librave_amd.so, checks the ABI)
    torch.ops.load_library(_TORCH_LIB)


def config_ints(cfg) -> List[int]:
    """rave_amd.config.RaveConfig -> the Engine constructor's flat int list
    (the rave_model_config fields in declaration order, leaky_slope apart)."""
    from . import _native as N
    c = N.model_config(cfg)
    out = [c.n_band, c.enc_bands, c.capacity, c.latent_size, c.kernel_size, c.speaker_size, c.n_ratios]
    out += list(c.ratios) + list(c.n_dilations) + [d for row in c.dilations for d in row]
    out += [c.amplitude_modulation, c.causal, c.activation, c.adain, c.conv_bias, c.convt_bias]
    out += [c.noise, c.noise_hidden, c.noise_bands, c.n_noise_ratios] + list(c.noise_ratios)
    out += [c.rvq_quantizers, c.rvq_codebook_size, c.fuse_units]
    return [int(v) for v in out]


class ScriptedRAVE(torch.nn.Module):
    """A scriptable nn~ module over the native engine (see the section comment).

    ``ScriptedRAVE(cfg, params, speaker, ...)`` takes the same inputs as
    rave_amd.RAVE; ``torch.jit.script(m)`` / ``m.export_to_ts(path)`` give a
    .ts whose engine re-creates itself on load (the weights travel inside)."""

    learn_target: Tuple[bool]
    reset_target: Tuple[bool]
    learn_source: Tuple[bool]
    reset_source: Tuple[bool]
    speaker: Tuple[int]
    record: Tuple[bool]
    is_using_adain: bool
    stereo: bool
    streaming: bool
    discrete: bool
    codebook_size: int
    hop: int
    latent_size: int
    active_speaker: int
    use_resampler: bool
    rs_ratio: int
    rs_down_pad: List[int]
    rs_up_pad: List[int]

    def __init__(self, cfg, params, speaker, hk=None, precision: str = "f32", stereo: bool = False,
                 streaming: Optional[bool] = None, block: int = 2048, speakers=None,
                 target_sr: Optional[int] = None, sampling_rate: int = 48000):
        """``speakers``: the embeddings the nn~ ``speaker`` attribute selects
        (speaker1..4 of scripts/export.py:84-93, e.g. SpeakerRAVE.embed outputs);
        index ``i`` picks ``speakers[i]``, any other index ``speaker5`` (the
        recorded target, ones until set, :96).  Default: ``[speaker]``.
        ``target_sr``: host rate; != sampling_rate adds the Resampler around
        the model (:101-106, 159-160, 331-332)."""
        super().__init__()
        import numpy as np
        from . import _native as N
        from . import pqmf as P
        load_torch_ops()
        self.streaming = bool(cfg.causal if streaming is None else streaming)
        self.discrete = cfg.rvq is not None
        self.codebook_size = int(cfg.rvq.codebook_size) if self.discrete else 0
        self.is_using_adain = bool(cfg.adain)
        if self.is_using_adain and stereo:
            raise ValueError("Stereo mode not yet supported with AdaIN")      # export.py:115-116
        self.stereo = bool(stereo)
        hk = P.design_bank(cfg.pqmf_attenuation, cfg.n_band) if hk is None else np.asarray(hk, np.float32)
        names = list(params) + ["pqmf.hk"]
        tensors = [torch.from_numpy(np.ascontiguousarray(params[k], np.float32)) for k in params]
        tensors.append(torch.from_numpy(np.ascontiguousarray(hk, np.float32)))
        spk = torch.from_numpy(np.ascontiguousarray(speaker, np.float32).reshape(-1))
        modes = {"auto": N.PREC_AUTO, "f32_tuned": N.PREC_F32_TUNED, "f32_bf3": N.PREC_F32_BF3,
                 "f32": N.PREC_F32, "split16": N.PREC_SPLIT16}
        if precision not in modes:
            raise ValueError(f"precision must be one of {sorted(modes)}")
        prec = modes[precision]
        self.engine = torch.classes.rave_amd.Engine(config_ints(cfg), float(cfg.leaky_slope), names, tensors, spk,
                                                    prec, int(block))
        self.hop = int(cfg.hop)
        # the encode method's channels: latents + speaker, or the RVQ indices
        self.latent_size = int(cfg.rvq.num_quantizers if self.discrete else cfg.latent_size + cfg.speaker_size)
        spks = [speaker] if speakers is None else list(speakers)
        self.register_buffer("speakers", torch.from_numpy(
            np.stack([np.asarray(e, np.float32).reshape(-1) for e in spks])) if spks else
            torch.zeros(0, int(cfg.speaker_size)))
        self.register_buffer("speaker5", torch.ones(int(cfg.speaker_size)))
        self.active_speaker = -1 if speakers is not None else 0
        # Resampler (rave/resampler.py) on torch.ops.rave_amd.fir
        self.use_resampler = target_sr is not None and int(target_sr) != int(sampling_rate)
        self.rs_ratio = 1
        self.rs_down_pad, self.rs_up_pad = [0, 0, 0], [0, 0, 0]
        self.register_buffer("rs_down_h", torch.zeros(1, 1))
        self.register_buffer("rs_up_h", torch.zeros(1, 1))
        self.register_buffer("rs_down_hist", torch.zeros(0, 0))
        self.register_buffer("rs_up_hist", torch.zeros(0, 0))
        if self.use_resampler:
            from . import resampler as R
            from .config import get_padding
            ratio, down, up = R.design(int(target_sr), int(sampling_rate))
            if self.streaming and ratio % 2:
                raise ValueError(f"When using streaming mode, resampling ratio must be a power of 2, got {ratio}")
            self.rs_ratio = ratio
            self.rs_down_h, self.rs_up_h = torch.from_numpy(down), torch.from_numpy(up)
            for pads, k, st in ((self.rs_down_pad, down.shape[1], ratio), (self.rs_up_pad, up.shape[1], 1)):
                l, r = get_padding(k, st, causal=cfg.causal)
                pads[0], pads[1], pads[2] = l, r, (st - r % st) % st     # + CachedConv1d's stride_delay
        io_ratio = self.hop * self.rs_ratio
        self.learn_target, self.reset_target = (False,), (False,)
        self.learn_source, self.reset_source = (False,), (False,)
        self.speaker, self.record = (0,), (False,)
        channels = ["(L)", "(R)"] if stereo else ["(mono)"]
        audio_in = ["(signal) Input audio signal"]
        audio_out = [f"(signal) Reconstructed audio signal {c}" for c in channels]
        latents = [f"(signal) Latent dimension {i}" for i in range(self.latent_size)]
        n_out = 2 if stereo else 1
        self._methods: List[str] = []
        self.register_method("encode", 1, 1, self.latent_size, io_ratio, audio_in, latents)
        self.register_method("decode", self.latent_size, io_ratio, n_out, 1, latents, audio_out)
        self.register_method("forward", 1, 1, n_out, 1, audio_in, audio_out)
        self._attributes: List[str] = ["learn_target", "reset_target", "learn_source", "reset_source",
                                       "speaker", "record"]

    @torch.jit.unused
    def register_method(self, name: str, in_channels: int, in_ratio: int, out_channels: int, out_ratio: int,
                        input_labels: List[str], output_labels: List[str]) -> None:
        """nn_tilde.Module.register_method: the method's metadata as buffers."""
        if len(input_labels) != in_channels or len(output_labels) != out_channels:
            raise ValueError(f"{name}: label counts must match the channel counts")
        self.register_buffer(f"{name}_params", torch.tensor([in_channels, in_ratio, out_channels, out_ratio]))
        setattr(self, f"{name}_input_labels", list(input_labels))
        setattr(self, f"{name}_output_labels", list(output_labels))
        self._methods.append(name)

    # ------------------------------------------------------------ nn~ metadata
    @torch.jit.export
    def get_methods(self) -> List[str]:
        return self._methods

    @torch.jit.export
    def get_method_params(self, method: str) -> List[int]:
        if method == "encode":
            return self.encode_params.tolist()
        if method == "decode":
            return self.decode_params.tolist()
        if method == "forward":
            return self.forward_params.tolist()
        raise ValueError("unknown method")

    @torch.jit.export
    def get_attributes(self) -> List[str]:
        return self._attributes

    @torch.jit.export
    def get_learn_target(self) -> bool:
        return self.learn_target[0]

    @torch.jit.export
    def set_learn_target(self, learn_target: bool) -> int:
        self.learn_target = (learn_target,)
        return 0

    @torch.jit.export
    def get_learn_source(self) -> bool:
        return self.learn_source[0]

    @torch.jit.export
    def set_learn_source(self, learn_source: bool) -> int:
        self.learn_source = (learn_source,)
        return 0

    @torch.jit.export
    def get_reset_target(self) -> bool:
        return self.reset_target[0]

    @torch.jit.export
    def set_reset_target(self, reset_target: bool) -> int:
        self.reset_target = (reset_target,)
        return 0

    @torch.jit.export
    def get_reset_source(self) -> bool:
        return self.reset_source[0]

    @torch.jit.export
    def set_reset_source(self, reset_source: bool) -> int:
        self.reset_source = (reset_source,)
        return 0

    @torch.jit.export
    def get_speaker(self) -> int:
        return self.speaker[0]

    @torch.jit.export
    def set_speaker(self, speaker: int) -> int:
        self.speaker = (speaker,)
        return 0

    @torch.jit.export
    def get_record(self) -> bool:
        return self.record[0]

    @torch.jit.export
    def set_record(self, record: bool) -> int:
        self.record = (record,)
        return 0

    # ------------------------------------------------------------ methods
    def update_adain(self) -> None:
        """ScriptedRAVE.update_adain (scripts/export.py:248-265)."""
        self.engine.adain_control(int(self.learn_source[0]), int(self.learn_target[0]), self.reset_source[0],
                                  self.reset_target[0])
        self.reset_source = (False,)
        self.reset_target = (False,)

    def _blocks(self, t: torch.Tensor, per_block: int) -> List[torch.Tensor]:
        T = t.shape[-1]
        if T % per_block != 0:
            raise ValueError("streaming buffers must be a multiple of the block")
        return [t[..., i:i + per_block] for i in range(0, T, per_block)]

    def _select_speaker(self) -> None:
        """scripts/export.py:384-396: the `speaker` attribute picks the embedding."""
        idx = self.speaker[0]
        if idx != self.active_speaker:
            if idx >= 0 and idx < self.speakers.shape[0]:
                self.engine.set_speaker(self.speakers[idx])
            else:
                self.engine.set_speaker(self.speaker5)
            self.active_speaker = idx

    def _fir(self, x: torch.Tensor, down: bool) -> torch.Tensor:
        """One Resampler conv on (B, 1, T); cached (streaming) or zero-padded."""
        h = self.rs_down_h if down else self.rs_up_h
        pads = self.rs_down_pad if down else self.rs_up_pad
        stride = self.rs_ratio if down else 1
        xs = x[:, 0, :].contiguous()
        if self.streaming:
            H = pads[0] + pads[1] + pads[2]
            hist = self.rs_down_hist if down else self.rs_up_hist
            if hist.shape[0] != xs.shape[0] or hist.shape[1] != H or hist.device != xs.device:
                hist = torch.zeros(xs.shape[0], H, device=xs.device)
                if down:
                    self.rs_down_hist = hist
                else:
                    self.rs_up_hist = hist
            y = torch.ops.rave_amd.fir(xs, h, stride, pads[0], pads[1], hist)
        else:
            y = torch.ops.rave_amd.fir(xs, h, stride, pads[0], pads[1], None)
        return y.unsqueeze(1)

    @torch.jit.export
    def encode(self, x: torch.Tensor) -> torch.Tensor:
        if self.is_using_adain:
            self.update_adain()
        self._select_speaker()
        if self.use_resampler:
            x = self._fir(x, True)                         # to_model_sampling_rate
        if self.discrete:       # DiscreteScriptedRAVE.post_process_latent: rvq.encode(z).float()
            if self.streaming:
                idx = torch.cat([self.engine.stream_encode_codes(b) for b in self._blocks(x, self.engine.block())], -1)
            else:
                idx = self.engine.encode_codes(x)
            return idx.float()
        if self.streaming:
            return torch.cat([self.engine.stream_encode(b) for b in self._blocks(x, self.engine.block())], -1)
        return self.engine.encode(x)

    @torch.jit.export
    def decode(self, z: torch.Tensor, from_forward: bool = False) -> torch.Tensor:
        if self.is_using_adain and not from_forward:
            self.update_adain()
        if self.stereo:
            z = torch.cat([z, z], 0)
        if self.discrete:       # pre_process_latent: clamp(z, 0, codebook_size - 1).long() -> rvq.decode
            idx = torch.clamp(z, 0, self.codebook_size - 1).long()
            if self.streaming:
                y = torch.cat([self.engine.stream_decode_codes(b)
                               for b in self._blocks(idx, self.engine.block() // self.hop)], -1)
            else:
                y = self.engine.decode_codes(idx)
        elif self.streaming:
            y = torch.cat([self.engine.stream_decode(b) for b in self._blocks(z, self.engine.block() // self.hop)], -1)
        else:
            y = self.engine.decode(z)
        if self.use_resampler:
            y = self._fir(y, False)                        # from_model_sampling_rate
        if self.stereo:
            y = torch.cat(y.chunk(2, 0), 1)
        return y

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.decode(self.encode(x), from_forward=True)

    @torch.jit.ignore
    def export_to_ts(self, path: str) -> None:
        """torch.jit.script + save (scripts/export.py:618)."""
        torch.jit.script(self).save(path)
