"""Operator-level drop-in for the cached_conv API the reference builds on.

The reference constructs every convolution through the ``cc.`` module
attribute at call time (rave/blocks.py:65,97,182,566; rave/__init__.py:14-27
makes them gin-configurable) and CachedPQMF wraps two ``cc.Conv1d``
(rave/pqmf.py:234-284).  ``cached_conv`` itself (cached-conv>=2.5.0,
requirements.txt:14) is third party and absent; its semantics are restated in
SURVEY.md section 8a rows 6-8.  This module keeps that constructor contract
over the HIP kernels (torch.ops.rave_amd.*, rave_amd/csrc/torch_ops.cpp over
the C-ABI), so a module tree written against ``cc`` runs on the MI355X:

* ``get_padding(kernel_size, stride=1, dilation=1, mode=None)`` -- p = (k-1)d+1,
  centred ((p-1)//2, p//2), causal (p-1, 0), k == 1 -> (0, 0);
* ``Conv1d(in, out, k, stride=, padding=(l, r), dilation=, bias=,
  cumulative_delay=)`` -- F.pad + conv offline; with ``use_cached_conv(True)``
  at construction the CachedConv1d form (an l + r input cache after a
  stride_delay crop-pad, ``cumulative_delay = (r + stride_delay + cd) // s``);
* ``ConvTranspose1d(in, out, 2r, stride=r, padding=r//2, bias=)`` -- torch's
  offline; cached: overlap-add of a 2*(r//2) cache, delay r//2 (the
  polyphase 2-tap form over one history column);
* ``CachedPadding1d``, ``AlignBranches``, ``CachedSequential`` -- delay
  bookkeeping (pure tensor ops);
* ``CachedPQMF(attenuation, n_band)`` -- forward (analysis + reverse_half) and
  inverse (reverse_half + polyphase synthesis), cached or not.

Weights live in ordinary ``weight`` / ``bias`` parameters (so
torch.nn.utils.weight_norm and the reference's state_dict names apply); the
kernels take a packed image made on first use (``prepare()`` re-packs after a
weight change; in eager Python a changed weight tensor is detected).
Everything here is TorchScript-scriptable: the custom ops are
``torch.ops.rave_amd.*``.  No CPU fallback: the ops need the GPU kernels.
"""
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from . import scripted as _scripted

_scripted.load_torch_ops()

MAX_BATCH_SIZE = 64
_USE_CACHED = False
_PAD_MODE = "centered"
_PRECISION = 0           # RAVE_PREC_F32; 1 = RAVE_PREC_SPLIT16 (include/rave_amd.h)
ACT_NONE, ACT_LEAKY, ACT_SNAKE = 0, 1, 2


def use_cached_conv(state: bool) -> None:
    """cc.use_cached_conv: modules built afterwards take their cached form."""
    global _USE_CACHED
    _USE_CACHED = bool(state)


def set_padding_mode(mode: str) -> None:
    """The gin binding ``cc.get_padding.mode`` (causal.gin:5)."""
    global _PAD_MODE
    if mode not in ("centered", "causal"):
        raise ValueError(mode)
    _PAD_MODE = mode


def set_precision(precision: str) -> None:
    """Arithmetic of the modules built afterwards: "f32" (exact fp32 MFMA) or
    "split16" (split-f16 GEMMs with the range guard)."""
    global _PRECISION
    _PRECISION = {"f32": 0, "split16": 1}[precision]


def get_padding(kernel_size: int, stride: int = 1, dilation: int = 1, mode: Optional[str] = None) -> Tuple[int, int]:
    mode = mode or _PAD_MODE
    if kernel_size == 1:
        return (0, 0)
    p = (kernel_size - 1) * dilation + 1
    if mode == "centered":
        return ((p - 1) // 2, p // 2)
    if mode == "causal":
        return (p - 1, 0)
    raise ValueError(mode)


class CachedPadding1d(nn.Module):
    """cached_conv's CachedPadding1d: prepend the last ``padding`` samples of the
    previous call (zeros at first); ``crop`` drops as many at the end (a pure
    delay line)."""

    def __init__(self, padding: int, crop: bool = False, channels: int = 0):
        super().__init__()
        self.padding = int(padding)
        self.crop = bool(crop)
        self.max_batch = MAX_BATCH_SIZE
        # runtime state, not a checkpoint entry (the reference registers it lazily)
        self.register_buffer("pad", torch.zeros(MAX_BATCH_SIZE, max(channels, 0), self.padding), persistent=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.padding == 0:
            return x
        if self.pad.shape[1] != x.shape[1] or self.pad.device != x.device:
            self.pad = torch.zeros(self.max_batch, x.shape[1], self.padding, device=x.device, dtype=x.dtype)
        # [pad | x] and the newest `padding` columns back into pad, on rave_copy
        return torch.ops.rave_amd.delay_line(x, self.pad, self.crop)


class _PackedConv(nn.Module):
    """Shared weight handling: torch-layout ``weight`` -> the kernels' packed image."""

    def __init__(self, c_in: int, c_out: int, kernel: int, stride: int, dilation: int, transposed: bool,
                 out_shift: int, bias: bool):
        super().__init__()
        self.c_in, self.c_out, self.kernel = int(c_in), int(c_out), int(kernel)
        self.stride, self.dilation = int(stride), int(dilation)
        self.transposed, self.out_shift = bool(transposed), int(out_shift)
        self.precision = _PRECISION
        shape = (c_in, c_out, kernel) if transposed else (c_out, c_in, kernel)
        ref = (nn.ConvTranspose1d(c_in, c_out, kernel, stride=stride) if transposed
               else nn.Conv1d(c_in, c_out, kernel, stride=stride, dilation=dilation))
        self.weight = nn.Parameter(ref.weight.detach().clone().reshape(shape))    # torch's default init
        self.bias = nn.Parameter(ref.bias.detach().clone()) if bias else None
        self.register_buffer("packed", torch.zeros(0), persistent=False)
        self.packed_key: List[int] = [0, 0]

    @torch.jit.export
    def fused(self) -> Tuple[int, float, Optional[torch.Tensor]]:
        """Not an activation (rave_amd.modules.FusedSequential's protocol)."""
        return 0, 0.0, None            # ACT_NONE

    @torch.jit.export
    def prepare(self) -> None:
        """Pack the current weight (after loading or changing it)."""
        w = self.weight
        p = torch.ops.rave_amd.pack_conv1d(w, self.c_in, self.c_out, self.kernel, self.stride, self.dilation,
                                           self.transposed, self.out_shift, self.precision)
        self.packed = p.to(w.device)

    def _packed_weight(self, x: torch.Tensor) -> torch.Tensor:
        if not torch.jit.is_scripting():
            key = [self.weight.data_ptr(), self.weight._version]
            if key != self.packed_key:           # weight replaced / modified (eager only)
                self.packed = torch.zeros(0)
                self.packed_key = key
        if self.packed.numel() == 0 or self.packed.device != x.device:
            self.prepare()
            self.packed = self.packed.to(x.device)
        return self.packed


class Conv1d(_PackedConv):
    """cc.Conv1d (offline: F.pad + conv; cached: CachedConv1d), fused on the
    kernels with an optional input activation (``activation``: ACT_LEAKY with
    ``slope`` or ACT_SNAKE with ``alpha``) and residual (``forward(x, res)``).
    ``forward(x, res, act, slope, alpha)`` with ``act >= 0`` takes the input
    activation of this call instead (the module tree fuses the activation
    module in front of each conv this way: rave_amd.modules)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1, padding=0,
                 dilation: int = 1, groups: int = 1, bias: bool = True, cumulative_delay: int = 0,
                 activation: int = ACT_NONE, slope: float = 0.2):
        if groups != 1:
            raise NotImplementedError("grouped convolutions are not on RAVE's path")
        super().__init__(in_channels, out_channels, kernel_size, stride, dilation, False, 0, bias)
        if isinstance(padding, int):
            pad = (int(padding), int(padding))
        else:
            pad = (int(padding[0]), int(padding[1]))
        self.pad_l, self.pad_r = pad
        self.act, self.slope = int(activation), float(slope)
        self.register_buffer("alpha", torch.ones(in_channels) if activation == ACT_SNAKE else torch.zeros(0),
                             persistent=False)
        self.cached = _USE_CACHED
        s = self.stride
        self.stride_delay = (s - ((self.pad_r + cumulative_delay) % s)) % s if self.cached else 0
        self.cumulative_delay = ((self.pad_r + self.stride_delay + cumulative_delay) // s) if self.cached else 0
        self.cache = CachedPadding1d(self.pad_l + self.pad_r, channels=in_channels)
        self.downsampling_delay = CachedPadding1d(self.stride_delay, crop=True, channels=in_channels)

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, act: int = -1, slope: float = 0.2,
                alpha: Optional[torch.Tensor] = None) -> torch.Tensor:
        packed = self._packed_weight(x)
        if act < 0:
            act, slope = self.act, self.slope
            alpha = self.alpha if self.act == 2 else None        # ACT_SNAKE
        if self.cached:
            x = self.cache(self.downsampling_delay(x))
            pl, pr = 0, 0
        else:
            pl, pr = self.pad_l, self.pad_r
        return torch.ops.rave_amd.conv1d(x.contiguous(), packed, self.bias, alpha, residual, self.c_out, self.kernel,
                                         self.stride, self.dilation, pl, pr, False, 0, act, slope, self.precision)


class ConvTranspose1d(_PackedConv):
    """cc.ConvTranspose1d(in, out, 2r, stride=r, padding=r//2): offline = torch's
    ConvTranspose1d; cached = CachedConvTranspose1d (overlap-add cache, output
    delayed by r//2 samples)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1, padding: int = 0,
                 output_padding: int = 0, groups: int = 1, bias: bool = False, dilation: int = 1,
                 cumulative_delay: int = 0, activation: int = ACT_NONE, slope: float = 0.2):
        if kernel_size != 2 * stride or padding != stride // 2 or output_padding or groups != 1 or dilation != 1:
            raise NotImplementedError("ConvTranspose1d: the kernels take kernel 2r, stride r, padding r//2")
        cached = _USE_CACHED
        super().__init__(in_channels, out_channels, kernel_size, stride, 1, True, 0 if cached else stride // 2, bias)
        self.cached = cached
        self.act, self.slope = int(activation), float(slope)
        self.register_buffer("alpha", torch.ones(in_channels) if activation == ACT_SNAKE else torch.zeros(0),
                             persistent=False)
        self.padding = int(padding)
        self.cumulative_delay = (self.padding + cumulative_delay * stride) if cached else 0
        self.hist = CachedPadding1d(1, channels=in_channels)    # the one input column the polyphase form reads back

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None, act: int = -1, slope: float = 0.2,
                alpha: Optional[torch.Tensor] = None) -> torch.Tensor:
        packed = self._packed_weight(x)
        if act < 0:
            act, slope = self.act, self.slope
            alpha = self.alpha if self.act == 2 else None        # ACT_SNAKE
        if self.cached:
            x = self.hist(x)
            pl = 1
        else:
            pl = 0
        return torch.ops.rave_amd.conv1d(x.contiguous(), packed, self.bias, alpha, residual, self.c_out, self.kernel,
                                         self.stride, 1, pl, 0, True, self.out_shift, act, slope, self.precision)


class AlignBranches(nn.Module):
    """cc.AlignBranches: delay each branch's input to max(delays)."""

    def __init__(self, *branches, delays: Optional[List[int]] = None, cumulative_delay: int = 0, stride: int = 1):
        super().__init__()
        self.branches = nn.ModuleList(branches)
        if delays is None:
            delays = [int(getattr(b, "cumulative_delay", 0)) for b in branches]
        max_delay = max(delays)
        self.paddings = nn.ModuleList([CachedPadding1d(max_delay - d, crop=True) for d in delays])
        self.cumulative_delay = int(cumulative_delay * stride) + max_delay

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        out: List[torch.Tensor] = []
        for b, p in zip(self.branches, self.paddings):
            out.append(b(p(x)))
        return out


class CachedSequential(nn.Sequential):
    """cc.CachedSequential: nn.Sequential carrying the last child's cumulative_delay."""

    def __init__(self, *args, cumulative_delay: int = 0, stride: int = 1):
        super().__init__(*args)
        self.cumulative_delay = int(cumulative_delay) * stride
        for m in reversed(list(self)):
            if hasattr(m, "cumulative_delay"):
                self.cumulative_delay += int(m.cumulative_delay)
                break


class CachedPQMF(nn.Module):
    """rave/pqmf.py:234-284 on the PQMF kernels: ``forward`` = analysis conv
    (k 513, stride n_band, padding get_padding(513)) + reverse_half (optionally
    only the first ``n_out`` bands, RAVE.encode's x[:, :6], rave/model.py:613);
    ``inverse`` = reverse_half + polyphase synthesis (k 33) * n_band + band
    flip + interleave.  Cached mode keeps taps-1 audio samples / frames."""

    def __init__(self, attenuation: float = 100.0, n_band: int = 16, hk=None):
        super().__init__()
        import numpy as np
        from . import pqmf as P
        hk = P.design_bank(attenuation, n_band) if hk is None else np.asarray(hk, np.float32)
        hkf, hki = P.kernels(hk)
        self.n_band = int(n_band)
        self.register_buffer("hk", torch.from_numpy(np.ascontiguousarray(hk, np.float32)))   # pqmf.hk
        self.register_buffer("hkf", torch.from_numpy(hkf), persistent=False)
        self.register_buffer("hki", torch.from_numpy(hki), persistent=False)
        self.cached = _USE_CACHED
        self.precision = _PRECISION
        self.pad_a = get_padding(int(hkf.shape[-1]))[0]
        self.pad_s = get_padding(int(hki.shape[-1]))[0]
        self.hist_a = CachedPadding1d(int(hkf.shape[-1]) - 1, channels=1)
        self.hist_s = CachedPadding1d(int(hki.shape[-1]) - 1, channels=self.n_band)
        self.hist_n = CachedPadding1d(int(hki.shape[-1]) - 1, channels=self.n_band)   # the epilogue's noise

    def forward(self, x: torch.Tensor, n_out: int = -1) -> torch.Tensor:
        n = self.n_band if n_out < 0 else n_out
        if self.cached:
            T = x.shape[-1]
            xc = self.hist_a(x).contiguous()
            # frame f of the cached conv starts at sample 16 f of [cache | block]
            y = torch.ops.rave_amd.pqmf_analysis(xc, self.hkf, n, 0, self.precision)
            return y[..., :T // self.n_band]
        return torch.ops.rave_amd.pqmf_analysis(x.contiguous(), self.hkf, n, self.pad_a, self.precision)

    def inverse(self, x: torch.Tensor, mode: int = 0, noise: Optional[torch.Tensor] = None) -> torch.Tensor:
        """mode 1 / 2: GeneratorV2's epilogue fused in front of the synthesis --
        x (B, 2 n_band, F) -> tanh(x[:n] sigmoid(x[n:]) + noise), or x (B, n_band,
        F) -> tanh(x + noise) (rave/blocks.py:699-707); cached mode keeps the
        history of x (and of noise) before the epilogue."""
        if self.cached:
            F = x.shape[-1]
            h = self.hist_s.padding
            xc = self.hist_s(x).contiguous()
            nc: Optional[torch.Tensor] = None
            if noise is not None:
                nc = self.hist_n(noise).contiguous()
            return torch.ops.rave_amd.pqmf_synthesis(xc, self.hki, 0, F, -h, self.precision, mode, nc)
        return torch.ops.rave_amd.pqmf_synthesis(x.contiguous(), self.hki, self.pad_s, 0, 0, self.precision, mode,
                                                 noise)


def adain(x: torch.Tensor, mean_x: torch.Tensor, std_x: torch.Tensor, mean_y: torch.Tensor, std_y: torch.Tensor,
          num_update_x: torch.Tensor, num_update_y: torch.Tensor, mode: int) -> torch.Tensor:
    """AdaptiveInstanceNormalization.forward, eval mode (rave/blocks.py:899-919):
    mode 0 transfer, 1 learn_x, 2 learn_y; updates the buffers in place."""
    return torch.ops.rave_amd.adain(x, mean_x, std_x, mean_y, std_y, num_update_x, num_update_y, mode)


def noise_synth(amp: torch.Tensor, u: torch.Tensor, n_band: int, noise_bands: int) -> torch.Tensor:
    """NoiseGeneratorV2's filter stage (rave/blocks.py:281-291): pre-sigmoid
    amplitudes (B, n_band noise_bands, F) and U[0,1) draws (B, F, n_band,
    target) -> filtered noise (B, n_band, F target)."""
    return torch.ops.rave_amd.noise_synth(amp, u, n_band, noise_bands)


def rvq_encode(z: torch.Tensor, codebooks: torch.Tensor) -> torch.Tensor:
    """ResidualVectorQuantization.encode (rave/quantization.py:302-310)."""
    return torch.ops.rave_amd.rvq_encode(z.contiguous(), codebooks)


def rvq_decode(idx: torch.Tensor, codebooks: torch.Tensor) -> torch.Tensor:
    """ResidualVectorQuantization.decode (rave/quantization.py:312-318)."""
    return torch.ops.rave_amd.rvq_decode(idx, codebooks)
