"""Block streaming of a causal model -- the cached_conv streaming mode.

``cc.use_cached_conv(True)`` (scripts/export.py:543, README.md:186-190;
cached_conv is the third-party ``cached-conv>=2.5.0``) turns every operator of
the causal graph into its cached form.  The native engine restates that on
the same kernels (include/rave_amd.h ``rave_stream_*``, rave_amd/csrc/
engine.cpp "streaming"): persistent ``[history | block]`` buffers per conv
input, the cached ConvTranspose1d as a polyphase 2-tap conv with one history
column, CachedPQMF's analysis / synthesis caches, NoiseGeneratorV2's cached
strided convs and per-frame filter, and AdaIN on each block's columns.

The decoder output equals one-shot causal decoding delayed by
sum(r//2 * upsampling) = 928 samples for v2 once the receptive field is
filled; the encoder is exact (zero delay).  State is created zeroed at
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
    """Per-block encode / decode of a causal RAVE with persistent caches."""

    def __init__(self, model: RAVE, batch: int = 1, block: int = 2048, graph: bool = True):
        cfg = model.cfg
        if not cfg.causal:
            raise ValueError("streaming requires a causal config (causal.gin)")
        if block % cfg.hop:
            raise ValueError(f"block must be a multiple of {cfg.hop}")
        self.model, self.cfg, self.B, self.block = model, cfg, batch, block
        self.Fz = block // cfg.hop
        self.F = block // cfg.n_band
        h = C.c_void_p()
        with torch.cuda.device(model.device):
            N.check(N.lib.rave_stream_create(model.handle, batch, block, N.STREAM_GRAPH if graph else 0,
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

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.decode(self.encode(x))

    @property
    def decode_delay(self) -> int:
        """Samples by which streamed decoding lags one-shot causal decoding."""
        return int(N.lib.rave_stream_delay(self.handle))
