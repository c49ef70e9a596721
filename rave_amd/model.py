"""``RAVE``: the reference's encode / decode / forward surface on the native engine.

Mirrors ``rave.model.RAVE`` (rave/model.py:594-634):

* ``encode(x)``  x (B, 1, T) -> PQMF analysis -> bands[:, :6] -> EncoderV2 ->
  cat(z, speaker) = (B, latent + 256, T / hop)          (model.py:594-622)
* ``decode(z)``  GeneratorV2 -> PQMF synthesis -> (B, 1, T)   (model.py:624-629)
* ``forward(x)`` = decode(encode(x))                          (model.py:631-634)

and, for the discrete config, the nn~ export path of DiscreteScriptedRAVE
(scripts/export.py:503-517): ``encode_codes`` (encoder -> rvq.encode) and
``decode_codes`` (rvq.decode -> cat speaker -> decoder -> PQMF inverse).

Everything below the call lives in the native engine (rave_amd/csrc/engine.cpp,
include/rave_amd.h ``rave_model_*``): the module graph, weight packing, launch
plans, the autotuner and every kernel launch.  This class converts the config
and the reference-named parameters, allocates outputs with torch and passes
torch's current stream.  There is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Mapping, Optional, Tuple

import numpy as np
import torch

from . import _native as N
from . import pqmf as P
from .adain import AdainState
from .config import RaveConfig
from .graph import build_graph
from .weights import check_params

# plan kinds of rave_model_plan_ops / rave_model_profile
ENCODE, DECODE, ENCODE_CODES, DECODE_CODES = 0, 1, 2, 3


def _stream(dev: torch.device) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


class RAVE:
    """HIP implementation of RAVE.encode / decode / forward for one config.

    ``precision``: "f32" (exact fp32 MFMA), "split16" (split-f16 GEMMs), or
    "auto" (per op the faster of the two, with every launch configuration,
    fused unit and residual stack timed at plan build), or "f32_tuned" (exact
    fp32 on every op, launch configurations and fused units timed as in auto), or
    "f32_bf3" (as f32_tuned, with the fused units also timed in bf16x3: fp32 on
    the bf16 matrix cores with an exact three-way operand split).  ``tuning`` replays the
    choices of an earlier model's ``tuning()`` without timing runs."""

    def __init__(self, cfg: RaveConfig, params: Mapping[str, np.ndarray], speaker: np.ndarray,
                 device=None, hk: Optional[np.ndarray] = None,
                 adain_stats: Optional[Mapping] = None, fuse_units: bool = True,
                 precision: str = "f32", tuning: Optional[list] = None):
        check_params(cfg, params)
        modes = {"auto": N.PREC_AUTO, "f32_tuned": N.PREC_F32_TUNED, "f32_bf3": N.PREC_F32_BF3,
                 "f32": N.PREC_F32, "split16": N.PREC_SPLIT16}
        if precision not in modes:
            raise ValueError(f"precision must be one of {sorted(modes)}")
        self.precision = precision
        self.cfg = cfg
        self.graph = build_graph(cfg)          # reference names (AdaIN modules, tests)
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise ValueError("rave_amd.RAVE runs on the GPU only (device must be cuda)")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.hk = P.design_bank(cfg.pqmf_attenuation, cfg.n_band) if hk is None else np.asarray(hk, np.float32)
        self.noise_target = int(np.prod(cfg.noise.ratios)) if cfg.noise is not None else 0
        spk = np.ascontiguousarray(np.asarray(speaker, np.float32).reshape(-1))
        if spk.size != cfg.speaker_size:
            raise ValueError(f"speaker embedding must have {cfg.speaker_size} values")
        ccfg = N.model_config(cfg)
        ccfg.fuse_units = int(fuse_units)
        keep = []
        plist = []
        for name, arr in list(params.items()) + [("pqmf.hk", self.hk)]:
            a = np.ascontiguousarray(np.asarray(arr, np.float32))
            keep.append(a)
            plist.append(N.Param(name.encode(), a.ctypes.data, a.size))
        parr = (N.Param * len(plist))(*plist)
        prec = modes[precision]
        h = C.c_void_p()
        with torch.cuda.device(self.device):
            N.check(N.lib.rave_model_create(C.byref(ccfg), parr, len(plist), spk.ctypes.data, prec, C.byref(h)),
                    "model_create")
        self.handle = h
        if tuning:
            self.set_tuning(tuning)
        self.adain: Optional[AdainState] = AdainState(self) if cfg.adain else None
        self._row0 = 0
        if adain_stats:
            if self.adain is None:
                raise ValueError("adain_stats given for a config without AdaIN")
            self.adain.load(adain_stats)

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and N is not None and N.lib is not None:
            N.lib.rave_model_destroy(h)
            self.handle = None

    # ------------------------------------------------------------ status
    def check(self, wait: bool = True) -> None:
        """Raise ``NativeError`` if a cooperative residual unit's in-launch
        hand-off gave up in a call that has run (its outputs are NaN); with
        ``wait`` the device's current stream is synchronised first, so every
        queued call is covered (rave_model_check).  encode / decode / forward
        also raise pending give-ups when they are called."""
        N.check(N.lib.rave_model_check(self.handle, int(bool(wait)), _stream(self.device)), "check")

    # ------------------------------------------------------------ tuning
    def tuning(self) -> list:
        """The autotuner's choices so far, JSON-serialisable; pass it back as
        ``RAVE(..., tuning=...)`` to build the same plans without timing runs."""
        n = N.lib.rave_model_tuning_get(self.handle, None, 0)
        if n < 0:
            N.check(n, "tuning_get")
        buf = C.create_string_buffer(n)
        N.lib.rave_model_tuning_get(self.handle, buf, n)
        out = []
        for line in buf.value.decode().splitlines():
            k, c, ms = line.split(" ")
            out.append([k, int(c), float(ms)])
        return out

    def set_tuning(self, tuning: list) -> None:
        text = "".join(f"{k if isinstance(k, str) else '|'.join(map(str, k))} {int(c)} {float(ms)!r}\n"
                       for k, c, ms in tuning)
        N.check(N.lib.rave_model_tuning_set(self.handle, text.encode()), "tuning_set")

    # ------------------------------------------------------------ speaker
    def set_speaker(self, embedding) -> None:
        """Replace the constant speaker embedding that encode / decode_codes
        concatenate (rave/model.py:617-618; the nn~ `speaker` choice among
        embeddings, scripts/export.py:384-396).  ``embedding``: speaker_size
        values, numpy or a torch tensor (e.g. ``SpeakerRAVE.embed`` output on
        this device).  Ordered on the current stream before later calls."""
        if isinstance(embedding, torch.Tensor):
            src = embedding.detach().to(self.device, torch.float32).contiguous().reshape(-1)
            if src.numel() != self.cfg.speaker_size:
                raise ValueError(f"speaker embedding must have {self.cfg.speaker_size} values")
            N.check(N.lib.rave_model_set_speaker(self.handle, src.data_ptr(), _stream(self.device)), "set_speaker")
            self._spk_keep = src          # the copy is asynchronous
            return
        spk = np.ascontiguousarray(np.asarray(embedding, np.float32).reshape(-1))
        if spk.size != self.cfg.speaker_size:
            raise ValueError(f"speaker embedding must have {self.cfg.speaker_size} values")
        src = torch.from_numpy(spk).to(self.device)
        N.check(N.lib.rave_model_set_speaker(self.handle, src.data_ptr(), _stream(self.device)), "set_speaker")
        self._spk_keep = src

    # ------------------------------------------------------------ AdaIN rows
    @property
    def adain_row0(self) -> int:
        """First AdaIN buffer row this process's batch uses (batch shards of a
        data-parallel job, rave/blocks.py:886-891)."""
        return self._row0

    @adain_row0.setter
    def adain_row0(self, v: int) -> None:
        N.check(N.lib.rave_model_set_row0(self.handle, int(v)), "set_row0")
        self._row0 = int(v)

    # ------------------------------------------------------------ measurement
    def ops(self, which: int, B: int, T: int) -> List[dict]:
        """Op list of one plan (built if needed): kind, precision, algorithmic
        FLOP and bytes, reference label."""
        with torch.cuda.device(self.device):
            n = N.lib.rave_model_plan_ops(self.handle, which, B, T, None, 0)
            if n < 0:
                N.check(n, "plan_ops")
            arr = (N.OpInfo * max(n, 1))()
            N.lib.rave_model_plan_ops(self.handle, which, B, T, arr, n)
        return [dict(kind=o.kind, precision=o.precision, flops=o.flops, bytes=o.bytes,
                     label=o.label.decode()) for o in arr[:n]]

    def profile(self, which: int, B: int, T: int, runs: int) -> None:
        """Arm per-op HIP-event timing of one plan for ``runs`` runs (0 disarms)."""
        N.check(N.lib.rave_model_profile(self.handle, which, B, T, int(runs)), "profile")

    def op_times(self, which: int, B: int, T: int) -> Tuple[np.ndarray, int]:
        """(per-op milliseconds summed over the recorded runs, runs)."""
        n = len(self.ops(which, B, T))
        buf = (C.c_float * max(n, 1))()
        runs = N.lib.rave_model_op_times(self.handle, which, B, T, buf, n)
        if runs < 0:
            N.check(runs, "op_times")
        return np.array(list(buf)[:n], np.float64), runs

    # ------------------------------------------------------------ public API
    def _check_audio(self, x: torch.Tensor) -> Tuple[int, int]:
        if not isinstance(x, torch.Tensor) or x.device.type != "cuda" or x.dtype != torch.float32:
            raise ValueError("x must be a float32 CUDA tensor")
        if x.dim() != 3 or x.shape[1] != 1:
            raise ValueError(f"x must be (B, 1, T), got {tuple(x.shape)}")
        B, _, T = x.shape
        if T % self.cfg.hop:
            raise ValueError(f"T={T} must be a multiple of {self.cfg.hop} (n_band * prod(ratios))")
        return B, T

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        B, T = self._check_audio(x)
        x = x.contiguous()
        z = torch.empty(B, self.cfg.latent_size + self.cfg.speaker_size, T // self.cfg.hop, device=x.device)
        with torch.cuda.device(x.device):
            N.check(N.lib.rave_model_encode(self.handle, x.data_ptr(), B, T, z.data_ptr(), _stream(x.device)),
                    "encode")
        return z

    def noise_shape(self, B: int, Fz: int) -> Tuple[int, int, int, int]:
        """Shape of NoiseGeneratorV2's uniform noise (torch.rand_like(ir),
        rave/blocks.py:287): (B, frames, n_band, target_size)."""
        F = Fz * self.cfg.hop // self.cfg.n_band
        return (B, F // self.noise_target, self.cfg.n_band, self.noise_target)

    def _noise(self, B: int, Fz: int, noise_u: Optional[torch.Tensor], dev) -> int:
        if self.cfg.noise is None:
            if noise_u is not None:
                raise ValueError("noise_u given for a config without a noise synthesizer")
            return 0
        if noise_u is None:
            return 0          # the engine draws U[0,1) on the device (rave_fill_uniform)
        shape = self.noise_shape(B, Fz)
        if noise_u.dtype != torch.float32 or noise_u.device.type != "cuda" or tuple(noise_u.shape) != shape:
            raise ValueError(f"noise_u must be a float32 CUDA tensor of shape {shape}")
        self._noise_keep = noise_u = noise_u.contiguous()
        return noise_u.data_ptr()

    def decode(self, z: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        """GeneratorV2 -> PQMF inverse.  For a noise config, ``noise_u`` (U[0,1),
        ``noise_shape``) replaces the reference's torch.rand_like draw; when
        omitted the engine draws it on the device."""
        if not isinstance(z, torch.Tensor) or z.device.type != "cuda" or z.dtype != torch.float32:
            raise ValueError("z must be a float32 CUDA tensor")
        if z.dim() != 3 or z.shape[1] != self.cfg.dec_in:
            raise ValueError(f"z must be (B, {self.cfg.dec_in}, T), got {tuple(z.shape)}")
        z = z.contiguous()
        B, _, Fz = z.shape
        y = torch.empty(B, 1, Fz * self.cfg.hop, device=z.device)
        u = self._noise(B, Fz, noise_u, z.device)
        with torch.cuda.device(z.device):
            N.check(N.lib.rave_model_decode(self.handle, z.data_ptr(), B, Fz, y.data_ptr(), u or None,
                                            _stream(z.device)), "decode")
        return y

    def forward(self, x: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self.decode(self.encode(x), noise_u)

    __call__ = forward

    def encode_codes(self, x: torch.Tensor) -> torch.Tensor:
        """encoder -> rvq.encode: (B, n_q, T/hop) int64 (discrete config)."""
        if self.cfg.rvq is None:
            raise ValueError("encode_codes needs a discrete (RVQ) config")
        B, T = self._check_audio(x)
        x = x.contiguous()
        idx = torch.empty(B, self.cfg.rvq.num_quantizers, T // self.cfg.hop, dtype=torch.int64, device=x.device)
        with torch.cuda.device(x.device):
            N.check(N.lib.rave_model_encode_codes(self.handle, x.data_ptr(), B, T, idx.data_ptr(),
                                                  _stream(x.device)), "encode_codes")
        return idx

    def decode_codes(self, idx: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        """rvq.decode (indices clamped as DiscreteScriptedRAVE) -> cat speaker ->
        decoder -> PQMF inverse."""
        if self.cfg.rvq is None:
            raise ValueError("decode_codes needs a discrete (RVQ) config")
        if idx.dtype != torch.int64 or idx.device.type != "cuda" or idx.dim() != 3 \
                or idx.shape[1] != self.cfg.rvq.num_quantizers:
            raise ValueError("idx must be an int64 CUDA tensor (B, n_q, T)")
        idx = idx.contiguous()
        B, _, Fz = idx.shape
        y = torch.empty(B, 1, Fz * self.cfg.hop, device=idx.device)
        u = self._noise(B, Fz, noise_u, idx.device)
        with torch.cuda.device(idx.device):
            N.check(N.lib.rave_model_decode_codes(self.handle, idx.data_ptr(), B, Fz, y.data_ptr(), u or None,
                                                  _stream(idx.device)), "decode_codes")
        return y

    def forward_codes(self, x: torch.Tensor) -> torch.Tensor:
        return self.decode_codes(self.encode_codes(x))
