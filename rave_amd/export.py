"""nn~ method surface over the HIP path.

Restates the host-side contract of ``ScriptedRAVE`` (scripts/export.py:58-480)
for a ``rave_amd.RAVE``:

* ``register_method(name, in_channels, in_ratio, out_channels, out_ratio,
  input_labels, output_labels)`` metadata (scripts/export.py:229-240), with the
  upstream-style ``encode`` / ``decode`` / ``forward`` registrations (the
  commented-out block at :172-227; the shipped ``myforward`` registration,
  :229-240, declares 2 input channels that v2's path does not take, SURVEY.md
  section 3);
* attributes through ``register_attribute`` and ``get_<name>`` / ``set_<name>``
  that store 1-tuples and return 0 from setters (:120-126, :427-479);
* ``encode`` (:298-314), ``decode`` with the stereo duplication (:317-336) and
  ``forward`` (:338-339), in streaming mode (cached_conv, one block per call;
  causal or centred padding) or offline (the default follows cfg.causal);
* a discrete config behaves as DiscreteScriptedRAVE (:503-517): ``encode``
  returns the RVQ indices as float, ``decode`` clamps and truncates them before
  rvq.decode.

nn~ itself loads a TorchScript module; the kernels here are reached through
ctypes, which TorchScript cannot script, so this is the method table and call
semantics an nn~ host would drive, not a ``torch.jit`` export.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

_ATTRIBUTES = (("learn_target", False), ("reset_target", False), ("learn_source", False),
               ("reset_source", False), ("speaker", 0), ("record", False))


class NNTildeRAVE:
    def __init__(self, model, stereo: bool = False, streaming: Optional[bool] = None,
                 block: int = 2048, batch: int = 1, speakers=None, target_sr: Optional[int] = None):
        """``speakers``: embeddings the ``speaker`` attribute selects (speaker1..4,
        scripts/export.py:84-93; any other index -> speaker5, ones, :96); None
        keeps the model's own.  ``target_sr``: host rate, wrapping the model in
        the Resampler (:101-106)."""
        cfg = model.cfg
        self.model, self.cfg, self.stereo = model, cfg, bool(stereo)
        self.streaming = cfg.causal if streaming is None else bool(streaming)
        if self.stereo and getattr(model, "adain", None) is not None:
            raise ValueError("Stereo mode not yet supported with AdaIN")      # export.py:115-116
        self.discrete = cfg.rvq is not None
        self.block, self.batch = block, batch
        self.sr = getattr(cfg, "sampling_rate", 48000)                       # v2.gin SAMPLING_RATE
        self.speakers = None if speakers is None else [torch.as_tensor(e, dtype=torch.float32).reshape(-1)
                                                       for e in speakers]
        self.speaker5 = torch.ones(cfg.speaker_size)
        self._active_speaker = 0 if speakers is None else -1
        self.resampler = None
        if target_sr is not None and int(target_sr) != self.sr:
            from rave_amd.resampler import Resampler
            self.resampler = Resampler(int(target_sr), self.sr, device=getattr(model, "device", None), causal=cfg.causal,
                                       streaming=self.streaming)
            self.sr = int(target_sr)
        # encode's channels: latents + speaker, or the RVQ indices (DiscreteScriptedRAVE)
        self.latent_size = cfg.rvq.num_quantizers if self.discrete else cfg.latent_size + cfg.speaker_size
        self._methods: Dict[str, Tuple[int, int, int, int, List[str], List[str]]] = {}
        self._attrs: Dict[str, tuple] = {}
        self._enc_stream = self._dec_stream = None
        for name, default in _ATTRIBUTES:
            self.register_attribute(name, default)
        ratio = cfg.hop * (self.resampler.ratio if self.resampler else 1)   # x_len // z.shape[-1]
        channels = ["(L)", "(R)"] if self.stereo else ["(mono)"]
        audio_in = ["(signal) Input audio signal"]
        audio_out = [f"(signal) Reconstructed audio signal {c}" for c in channels]
        latents = [f"(signal) Latent dimension {i}" for i in range(self.latent_size)]
        n_out = 2 if self.stereo else 1
        self.register_method("encode", 1, 1, self.latent_size, ratio, audio_in, latents)
        self.register_method("decode", self.latent_size, ratio, n_out, 1, latents, audio_out)
        self.register_method("forward", 1, 1, n_out, 1, audio_in, audio_out)

    # ------------------------------------------------------------ nn~ metadata
    def register_method(self, name: str, in_channels: int, in_ratio: int, out_channels: int,
                        out_ratio: int, input_labels: List[str], output_labels: List[str]) -> None:
        if len(input_labels) != in_channels or len(output_labels) != out_channels:
            raise ValueError(f"{name}: label counts must match the channel counts")
        self._methods[name] = (in_channels, in_ratio, out_channels, out_ratio,
                               list(input_labels), list(output_labels))

    def get_methods(self) -> List[str]:
        return list(self._methods)

    def get_method_params(self, name: str) -> List[int]:
        """[in_channels, in_ratio, out_channels, out_ratio], as nn~ queries them."""
        return list(self._methods[name][:4])

    def get_method_labels(self, name: str) -> Tuple[List[str], List[str]]:
        return self._methods[name][4], self._methods[name][5]

    def register_attribute(self, name: str, default) -> None:
        self._attrs[name] = (default,)

    def get_attributes(self) -> List[str]:
        return list(self._attrs)

    def get_attribute(self, name: str):
        return self._attrs[name][0]

    def set_attribute(self, name: str, value) -> int:
        """Store ``value`` as a 1-tuple.  Bool attributes take a bool, an int 0/1
        or a 0-d tensor; int attributes an int or 0-d integer tensor.  Anything
        else (e.g. the string 'False', which bool() would turn True) raises."""
        if name not in self._attrs:
            raise KeyError(name)
        if isinstance(value, tuple) and len(value) == 1:
            value = value[0]
        if isinstance(value, torch.Tensor):
            if value.numel() != 1:
                raise TypeError(f"{name}: expected a scalar, got a tensor of shape {tuple(value.shape)}")
            value = value.item()
        default = self._attrs[name][0]
        if isinstance(default, bool):
            if isinstance(value, bool):
                pass
            elif isinstance(value, int) and value in (0, 1):
                value = bool(value)
            else:
                raise TypeError(f"{name}: expected a bool, got {value!r}")
        elif isinstance(default, int):
            if isinstance(value, bool) or not isinstance(value, int):
                if isinstance(value, float) and value.is_integer():
                    value = int(value)
                else:
                    raise TypeError(f"{name}: expected an int, got {value!r}")
        self._attrs[name] = (value,)
        return 0

    def __getattr__(self, item: str):
        # get_<attr> / set_<attr>, the @torch.jit.export accessors of export.py:427-479
        attrs = self.__dict__.get("_attrs", {})
        if item.startswith("get_") and item[4:] in attrs:
            return lambda: self.get_attribute(item[4:])
        if item.startswith("set_") and item[4:] in attrs:
            return lambda v: self.set_attribute(item[4:], v)
        raise AttributeError(item)

    # ------------------------------------------------------------ AdaIN controls
    def update_adain(self) -> None:
        """ScriptedRAVE.update_adain (scripts/export.py:248-265): the learn
        flags of every AdaIN module follow learn_target / learn_source, a set
        reset_* flag resets that side's statistics once and is cleared."""
        ad = getattr(self.model, "adain", None)
        if ad is None:
            return
        ad.set_learn(learn_x=self.get_attribute("learn_source"), learn_y=self.get_attribute("learn_target"))
        if self.get_attribute("reset_target"):
            ad.reset_y()
        if self.get_attribute("reset_source"):
            ad.reset_x()
        self._attrs["reset_source"] = (False,)
        self._attrs["reset_target"] = (False,)

    def _select_speaker(self) -> None:
        """scripts/export.py:384-396: the ``speaker`` attribute picks the
        embedding encode concatenates (set on the model when it changes)."""
        if self.speakers is None:
            return
        idx = self.get_attribute("speaker")
        if idx != self._active_speaker:
            emb = self.speakers[idx] if 0 <= idx < len(self.speakers) else self.speaker5
            self.model.set_speaker(emb)
            self._active_speaker = idx

    # ------------------------------------------------------------ methods
    def _enc_streamer(self, batch: int):
        """The encode stream; created (zeroed) on first use or a batch change,
        without touching the decode stream's caches."""
        from rave_amd.streaming import StreamingRAVE
        if self._enc_stream is None or self._enc_stream.B != batch:
            self._enc_stream = StreamingRAVE(self.model, batch=batch, block=self.block, direction="encode")
        return self._enc_stream

    def _dec_streamer(self, batch: int):
        from rave_amd.streaming import StreamingRAVE
        if self._dec_stream is None or self._dec_stream.B != batch:
            self._dec_stream = StreamingRAVE(self.model, batch=batch, block=self.block, direction="decode")
        return self._dec_stream

    def _blocks(self, t: torch.Tensor, per_block: int) -> List[torch.Tensor]:
        """Split a host buffer into the stream's blocks (any multiple of the
        block length is accepted, as cached_conv accepts any multiple of hop
        once the plan's block is fixed)."""
        T = t.shape[-1]
        if T % per_block:
            raise ValueError(f"streaming buffers must be a multiple of the block: {T} columns, "
                             f"block {per_block} (configure NNTildeRAVE(block=...))")
        return [t[..., i:i + per_block].contiguous() for i in range(0, T, per_block)]

    def _check(self, name: str, t: torch.Tensor) -> None:
        c = self._methods[name][0]
        if t.dim() != 3 or t.shape[1] != c:
            raise ValueError(f"{name}: expected (B, {c}, T), got {tuple(t.shape)}")

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        """scripts/export.py:298-314 (update_adain -> PQMF -> encoder on 6 bands
        -> cat speaker)."""
        self._check("encode", x)
        self.update_adain()
        self._select_speaker()
        if self.resampler is not None:
            x = self.resampler.to_model_sampling_rate(x)
        if self.discrete:        # post_process_latent: rvq.encode(z).float()
            if self.streaming:
                st = self._enc_streamer(x.shape[0])
                idx = torch.cat([st.encode_codes(b) for b in self._blocks(x, self.block)], -1)
            else:
                idx = self.model.encode_codes(x)
            return idx.float()
        if self.streaming:
            st = self._enc_streamer(x.shape[0])
            return torch.cat([st.encode(b) for b in self._blocks(x, self.block)], -1)
        return self.model.encode(x)

    def decode(self, z: torch.Tensor, from_forward: bool = False) -> torch.Tensor:
        """scripts/export.py:317-336: update_adain unless called from forward;
        stereo decodes the batch twice and puts the copies side by side as
        channels (L, R)."""
        self._check("decode", z)
        if not from_forward:
            self.update_adain()
        if self.stereo:
            z = torch.cat([z, z], 0)
        if self.discrete:        # pre_process_latent: clamp(z, 0, codebook_size - 1).long()
            idx = torch.clamp(z, 0, self.cfg.rvq.codebook_size - 1).long()
            if self.streaming:
                st = self._dec_streamer(idx.shape[0])
                y = torch.cat([st.decode_codes(b) for b in self._blocks(idx, self.block // self.cfg.hop)], -1)
            else:
                y = self.model.decode_codes(idx)
        elif self.streaming:
            st = self._dec_streamer(z.shape[0])
            y = torch.cat([st.decode(b) for b in self._blocks(z, self.block // self.cfg.hop)], -1)
        else:
            y = self.model.decode(z)
        if self.resampler is not None:
            y = self.resampler.from_model_sampling_rate(y)
        if self.stereo:
            y = torch.cat(y.chunk(2, 0), 1)
        return y

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.decode(self.encode(x), from_forward=True)

    __call__ = forward

    def reset(self) -> None:
        """Zero the streaming caches (a fresh nn~ instance)."""
        for s in (self._enc_stream, self._dec_stream):
            if s is not None:
                s.reset()
        if self.resampler is not None:
            self.resampler.reset()


# The TorchScript (nn~ .ts) export lives in rave_amd/scripted.py (no postponed
# annotations there: TorchScript resolves attribute annotations at script time).
