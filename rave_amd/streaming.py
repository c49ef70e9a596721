"""Block streaming -- the cached_conv streaming mode, causal or centred.

``cc.use_cached_conv(True)`` (scripts/export.py:543, README.md:186-190;
cached_conv is the third-party ``cached-conv>=2.5.0``) turns every operator of
the causal graph into its cached form.  The native engine restates that on
the same kernels (include/rave_amd.h ``rave_stream_*``, rave_amd/csrc/
engine.cpp "streaming"): persistent ``[history | block]`` buffers per conv
input, the cached ConvTranspose1d as a polyphase 2-tap conv with one history
column, CachedPQMF's analysis / synthesis caches, NoiseGeneratorV2's cached
strided convs and per-frame filter, and AdaIN on each block's columns.

Centred (non-causal) configs stream the way the reference's default model
exports with ``--streaming`` (README.md:187-190): every CachedConv1d reads an
(l + r)-column cache, so it lags its offline conv by r, and Residual's
AlignBranches delays the identity branch by the unit's delay
(rave/blocks.py:32-46).  The decoder output equals one-shot decoding delayed
by ``decode_delay`` samples (928 for v2 causal, 13280 for v2 centred) once the
receptive field is filled; a causal encoder is exact (zero delay), a centred
one decimates its delayed signal on the strided convs' own phase, as the
reference's does.  Discrete configs stream RVQ indices (``encode_codes`` /
``decode_codes``, DiscreteScriptedRAVE).  State is created zeroed at
construction (the reference creates it lazily on the first call) and is not
re-entrant: one StreamingRAVE per stream, like one nn~ instance.  With
``graph=True`` every block replays a captured hipGraph.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from . import _native as N
from .model import RAVE, _stream


class StreamingRAVE:
    """Per-block encode / decode of a RAVE with persistent caches.
    ``direction``: "both", "encode" or "decode" (build one side only)."""

    def __init__(self, model: RAVE, batch: int = 1, block: int = 2048, graph: bool = True,
                 direction: str = "both"):
        cfg = model.cfg
        if block % cfg.hop:
            raise ValueError(f"block must be a multiple of {cfg.hop}")
        flags = {"both": 0, "encode": N.STREAM_ENCODE_ONLY, "decode": N.STREAM_DECODE_ONLY}
        if direction not in flags:
            raise ValueError(f"direction must be one of {sorted(flags)}")
        self.model, self.cfg, self.B, self.block = model, cfg, batch, block
        self.Fz = block // cfg.hop
        self.F = block // cfg.n_band
        h = C.c_void_p()
        with torch.cuda.device(model.device):
            N.check(N.lib.rave_stream_create(model.handle, batch, block,
                                             (N.STREAM_GRAPH if graph else 0) | flags[direction],
                                             C.byref(h)), "stream_create")
        self.handle = h

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and N is not None and N.lib is not None:
            N.lib.rave_stream_destroy(h)
            self.handle = None

    def reset(self) -> None:
        """Zero every cache (the reference's freshly created CachedPadding1d)."""
        N.check(N.lib.rave_stream_reset(self.handle, _stream(self.model.device)), "stream_reset")

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        if tuple(x.shape) != (self.B, 1, self.block) or x.dtype != torch.float32 or x.device.type != "cuda":
            raise ValueError(f"x must be a float32 CUDA tensor of shape {(self.B, 1, self.block)}")
        x = x.contiguous()
        z = torch.empty(self.B, self.cfg.latent_size + self.cfg.speaker_size, self.Fz, device=x.device)
        with torch.cuda.device(x.device):
            N.check(N.lib.rave_stream_encode(self.handle, x.data_ptr(), z.data_ptr(), _stream(x.device)),
                    "stream_encode")
        return z

    def decode(self, z: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        if tuple(z.shape) != (self.B, self.cfg.dec_in, self.Fz) or z.dtype != torch.float32 \
                or z.device.type != "cuda":
            raise ValueError(f"z must be a float32 CUDA tensor of shape {(self.B, self.cfg.dec_in, self.Fz)}")
        z = z.contiguous()
        y = torch.empty(self.B, 1, self.block, device=z.device)
        u = None
        if noise_u is not None:
            if self.cfg.noise is None:
                raise ValueError("noise_u given for a config without a noise synthesizer")
            shape = self.model.noise_shape(self.B, self.Fz)
            if tuple(noise_u.shape) != shape or noise_u.dtype != torch.float32 or noise_u.device.type != "cuda":
                raise ValueError(f"noise_u must be a float32 CUDA tensor of shape {shape}")
            noise_u = noise_u.contiguous()
            u = noise_u.data_ptr()
        with torch.cuda.device(z.device):
            N.check(N.lib.rave_stream_decode(self.handle, z.data_ptr(), y.data_ptr(), u, _stream(z.device)),
                    "stream_decode")
        return y

    def _noise_arg(self, noise_u):
        if noise_u is None:
            return None
        if self.cfg.noise is None:
            raise ValueError("noise_u given for a config without a noise synthesizer")
        shape = self.model.noise_shape(self.B, self.Fz)
        if tuple(noise_u.shape) != shape or noise_u.dtype != torch.float32 or noise_u.device.type != "cuda":
            raise ValueError(f"noise_u must be a float32 CUDA tensor of shape {shape}")
        return noise_u.contiguous()

    def encode_codes(self, x: torch.Tensor) -> torch.Tensor:
        """One block -> RVQ indices (B, n_q, block / hop) int64 (discrete config)."""
        if self.cfg.rvq is None:
            raise ValueError("encode_codes needs a discrete (RVQ) config")
        if tuple(x.shape) != (self.B, 1, self.block) or x.dtype != torch.float32 or x.device.type != "cuda":
            raise ValueError(f"x must be a float32 CUDA tensor of shape {(self.B, 1, self.block)}")
        x = x.contiguous()
        idx = torch.empty(self.B, self.cfg.rvq.num_quantizers, self.Fz, dtype=torch.int64, device=x.device)
        with torch.cuda.device(x.device):
            N.check(N.lib.rave_stream_encode_codes(self.handle, x.data_ptr(), idx.data_ptr(), _stream(x.device)),
                    "stream_encode_codes")
        return idx

    def decode_codes(self, idx: torch.Tensor, noise_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One block of RVQ indices (clamped to the codebook) -> audio (B, 1, block)."""
        if self.cfg.rvq is None:
            raise ValueError("decode_codes needs a discrete (RVQ) config")
        shape = (self.B, self.cfg.rvq.num_quantizers, self.Fz)
        if tuple(idx.shape) != shape or idx.dtype != torch.int64 or idx.device.type != "cuda":
            raise ValueError(f"idx must be an int64 CUDA tensor of shape {shape}")
        idx = idx.contiguous()
        u = self._noise_arg(noise_u)
        y = torch.empty(self.B, 1, self.block, device=idx.device)
        with torch.cuda.device(idx.device):
            N.check(N.lib.rave_stream_decode_codes(self.handle, idx.data_ptr(), y.data_ptr(),
                                                   None if u is None else u.data_ptr(), _stream(idx.device)),
                    "stream_decode_codes")
        return y

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.cfg.rvq is not None:
            return self.decode_codes(self.encode_codes(x))
        return self.decode(self.encode(x))

    @property
    def decode_delay(self) -> int:
        """Samples by which streamed decoding lags one-shot decoding."""
        return int(N.lib.rave_stream_delay(self.handle))

    def launches(self, which: str = "decode") -> int:
        """Kernel launches of one block ("encode" or "decode"): the captured
        graph's kernel nodes (graph mode) or the plan's launches (eager: one
        per op, a run of history shifts going out as one batched launch)."""
        n = int(N.lib.rave_stream_launches(self.handle, {"encode": 0, "decode": 1}[which]))
        if n < 0:
            N.check(n, "stream_launches")
        return n
