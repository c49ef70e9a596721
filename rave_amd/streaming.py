"""Block streaming of a causal model -- the cached_conv streaming mode.

Restates what ``cc.use_cached_conv(True)`` does to every operator of the
causal v2 graph (scripts/export.py:543, README.md:186-190; cached_conv is the
third-party ``cached-conv>=2.5.0``), without changing any kernel:

* a causal Conv1d with padding (p-1, 0) keeps the last p-1 samples of its input
  (CachedPadding1d).  Here each conv input is a persistent buffer
  ``[history | block]``; the conv reads it with zero padding 0, and after the
  block the newest ``history`` columns are moved to the front (SHIFT_HISTORY).
  The cached values are pre-activation (the activation is fused into the conv
  prologue; act(0) = 0 keeps the zero start state identical);
* CachedConvTranspose1d (overlap-add of a 2*(r//2) cache) is the polyphase
  2-tap conv with one input history column and no output crop;
* CachedPQMF: analysis keeps 512 audio samples, synthesis 32 frames;
* Residual/AlignBranches delays are 0 in causal mode (conv cumulative delays
  are 0), so residual adds read the block columns directly.

The decoder output equals one-shot causal decoding delayed by
sum(r//2 * upsampling) = 928 samples for v2 once the receptive field is
filled; the encoder is exact (zero delay).  State is created zeroed at
construction (the reference creates it lazily on the first call) and is not
re-entrant: one StreamingRAVE per stream, like one nn~ instance.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import _native as N
from .config import get_padding
from .graph import ConvNode
from .model import RAVE, Plan, View, splitk_floats


def _need(n: ConvNode) -> int:
    """History columns a streaming conv needs on its input."""
    if n.transposed:
        return 1
    if n.pad[1] != 0:
        raise ValueError(f"{n.name}: streaming needs causal padding, got {n.pad}")
    return n.pad[0]


class StreamingRAVE:
    """Per-block encode / decode of a causal RAVE with persistent caches."""

    def __init__(self, model: RAVE, batch: int = 1, block: int = 2048):
        cfg = model.cfg
        if not cfg.causal:
            raise ValueError("streaming requires a causal config (causal.gin)")
        if cfg.noise is not None:
            raise NotImplementedError("streaming noise synthesis is not implemented")
        if model.adain is not None and model.adain.active:
            raise NotImplementedError("streaming with learned AdaIN statistics is not implemented "
                                      "(the identity AdaIN of a fresh model is)")
        if block % cfg.hop:
            raise ValueError(f"block must be a multiple of {cfg.hop}")
        self.model, self.cfg, self.B, self.block = model, cfg, batch, block
        self.Fz = block // cfg.hop
        self.F = block // cfg.n_band
        self._enc = self._build_encoder()
        self._dec = self._build_decoder()
        self.reset()

    # ---------------------------------------------------------------- building
    def _buffers(self, plan: Plan, nodes: List[ConvNode], sizes: Dict[str, Tuple[int, int]],
                 extra_need: Dict[str, int]) -> Dict[str, Tuple[View, int, int]]:
        """Persistent [history | block] buffers for every tensor of ``nodes``.
        sizes: tensor -> (channels, block columns)."""
        need: Dict[str, int] = dict(extra_need)
        for n in nodes:
            need[n.src] = max(need.get(n.src, 0), _need(n))
        bufs = {}
        B = self.B
        for name, (c, t) in sizes.items():
            h = need.get(name, 0)
            width = h + t
            off = plan.ws.alloc(B * c * width)
            bufs[name] = (View("ws", off, c * width, width), h, t)
        return bufs

    def _conv_stream(self, plan: Plan, n: ConvNode, bufs) -> None:
        m = self.model
        src, h_src, t_src = bufs[n.src]
        dst, h_dst, t_dst = bufs[n.dst]
        need = _need(n)
        x = View("ws", src.off + (h_src - need), src.sb, src.sc)
        y = View(dst.slot, dst.off + h_dst, dst.sb, dst.sc) if dst.slot == "ws" else dst
        res = None
        if n.residual:
            r, h_r, _ = bufs[n.residual]
            res = View("ws", r.off + h_r, r.sb, r.sc)
        _, bo, ao = m.w_off[n.name]
        t_in = need + t_src
        s = dict(c_in=n.c_in, c_out=n.c_out, kernel=n.kernel, stride=n.stride, dilation=n.dilation,
                 pad_left=1 if n.transposed else 0, pad_right=0, transposed=int(n.transposed),
                 out_shift=0,
                 act=N.ACT[n.act], leaky_slope=self.cfg.leaky_slope, batch=self.B, t_in=t_in,
                 t_out=t_dst, x_sb=x.sb, x_sc=x.sc, y_sb=y.sb, y_sc=y.sc,
                 r_sb=res.sb if res else 0, r_sc=res.sc if res else 0)
        ptrs = dict(x=x, y=y, residual=res,
                    bias=View("arena", bo, 0, 0) if bo is not None else None,
                    alpha=View("arena", ao, 0, 0) if ao is not None else None)
        pr, cfg = m.conv_launch(n, s, ptrs, stream_form=n.transposed)
        s["precision"], s["config"] = pr, cfg
        # ConvTranspose: packed for the cached form (out_shift 0)
        pack = m.w_pack_stream if n.transposed else m.w_pack
        ptrs["weight"] = View("arena", pack[(n.name, pr)], 0, 0)
        ptrs["partial"] = plan.splitk_view(splitk_floats(s, res is not None))
        plan.add(N.OP_CONV, N.ConvArgs, s, ptrs, label=n.name)

    def _shift_all(self, plan: Plan, bufs) -> None:
        for name, (v, h, t) in bufs.items():
            if h > 0 and v.slot == "ws":
                c = v.sb // v.sc
                plan.add(N.OP_SHIFT_HISTORY, N.ShiftArgs,
                         dict(batch=self.B, channels=c, hist=h, t_new=t, sb=v.sb, sc=v.sc),
                         dict(buf=v), label=f"shift:{name}")

    def _tensor_sizes(self, nodes: List[ConvNode], first: str, c0: int, t0: int):
        sizes = {first: (c0, t0)}
        for n in nodes:
            t_in = sizes[n.src][1]
            t_out = t_in * n.stride if n.transposed else t_in // n.stride
            sizes[n.dst] = (n.c_out, t_out)
        return sizes

    def _build_encoder(self) -> Plan:
        cfg, m, B = self.cfg, self.model, self.B
        plan = Plan(m.arena)
        nodes = m.graph.encoder
        sizes = {"audio": (1, self.block)}
        sizes.update(self._tensor_sizes(nodes, "enc_in", cfg.enc_bands, self.F))
        sizes.pop("latent")
        hist_audio = m.taps_a - 1                               # 512
        bufs = self._buffers(plan, nodes, sizes, {"audio": hist_audio})
        zc = cfg.latent_size + cfg.speaker_size
        bufs["latent"] = (View(1, 0, zc * self.Fz, self.Fz), 0, self.Fz)
        a, ha, ta = bufs["audio"]
        plan.add(N.OP_COPY, N.CopyArgs,
                 dict(batch=B, channels=1, t_len=self.block, x_sb=self.block, x_sc=self.block,
                      y_sb=a.sb, y_sc=a.sc),
                 dict(x=View(0, 0, self.block, self.block), y=View("ws", a.off + ha, a.sb, a.sc)))
        e, he, _ = bufs["enc_in"]
        plan.add(N.OP_PQMF_ANALYSIS, N.AnalysisArgs,
                 dict(n_band=cfg.n_band, taps=m.taps_a, n_out_bands=cfg.enc_bands, batch=B,
                      t_in=ha + self.block, pad_left=0, t_out=self.F, x_sb=a.sb, y_sb=e.sb, y_sc=e.sc),
                 dict(x=View("ws", a.off, a.sb, a.sc), y=View("ws", e.off + he, e.sb, e.sc),
                      hkf=View("arena", m.hkf_off, 0, 0)))
        for n in nodes:
            self._conv_stream(plan, n, bufs)
        m._fill_speaker(plan, B, self.Fz, View(1, cfg.latent_size * self.Fz, zc * self.Fz, self.Fz))
        self._shift_all(plan, bufs)
        self._enc_bufs = bufs
        return plan.finalize(m.device)

    def _build_decoder(self) -> Plan:
        cfg, m, B = self.cfg, self.model, self.B
        plan = Plan(m.arena)
        nodes = m.graph.decoder
        sizes = self._tensor_sizes(nodes, "dec_in", cfg.dec_in, self.Fz)
        hist_wave = m.taps_s - 1                                # 32 frames
        bufs = self._buffers(plan, nodes, sizes, {"wave": hist_wave})
        z, hz, _ = bufs["dec_in"]
        plan.add(N.OP_COPY, N.CopyArgs,
                 dict(batch=B, channels=cfg.dec_in, t_len=self.Fz, x_sb=cfg.dec_in * self.Fz,
                      x_sc=self.Fz, y_sb=z.sb, y_sc=z.sc),
                 dict(x=View(0, 0, cfg.dec_in * self.Fz, self.Fz), y=View("ws", z.off + hz, z.sb, z.sc)))
        for n in nodes:
            self._conv_stream(plan, n, bufs)
        w, hw, tw = bufs["wave"]
        plan.add(N.OP_PQMF_SYNTHESIS, N.SynthesisArgs,
                 dict(n_band=cfg.n_band, taps=m.taps_s, batch=B, t_in=self.F, pad_left=0,
                      mode=1 if cfg.amplitude_modulation else 2, frame0=-hw, x_len=hw + self.F,
                      x_sb=w.sb, x_sc=w.sc, n_sb=0, n_sc=0, y_sb=self.block),
                 dict(x=View("ws", w.off, w.sb, w.sc), y=View(1, 0, self.block, self.block),
                      noise=None, hki=View("arena", m.hki_off, 0, 0)))
        self._shift_all(plan, bufs)
        self._dec_bufs = bufs
        return plan.finalize(m.device)

    # ---------------------------------------------------------------- API
    def reset(self) -> None:
        """Zero every cache (the reference's freshly created CachedPadding1d)."""
        self._enc.ws_tensor.zero_()
        self._dec.ws_tensor.zero_()

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        if tuple(x.shape) != (self.B, 1, self.block) or x.dtype != torch.float32 or x.device.type != "cuda":
            raise ValueError(f"x must be a float32 CUDA tensor of shape {(self.B, 1, self.block)}")
        x = x.contiguous()
        z = torch.empty(self.B, self.cfg.latent_size + self.cfg.speaker_size, self.Fz, device=x.device)
        self._enc.run([x.data_ptr(), z.data_ptr()])
        return z

    def decode(self, z: torch.Tensor) -> torch.Tensor:
        if tuple(z.shape) != (self.B, self.cfg.dec_in, self.Fz) or z.dtype != torch.float32 \
                or z.device.type != "cuda":
            raise ValueError(f"z must be a float32 CUDA tensor of shape {(self.B, self.cfg.dec_in, self.Fz)}")
        z = z.contiguous()
        y = torch.empty(self.B, 1, self.block, device=z.device)
        self._dec.run([z.data_ptr(), y.data_ptr()])
        return y

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.decode(self.encode(x))

    @property
    def decode_delay(self) -> int:
        """Samples by which streamed decoding lags one-shot causal decoding."""
        d, up = 0, self.cfg.hop
        for r in self.cfg.ratios[::-1]:
            up //= r
            d += (r // 2) * up
        return d
